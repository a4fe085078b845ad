"""aigar_amd -- MI355X-native agar.io environment stepper.

Replaces the reference `src/model` hot path (Field.update() tick and
Bot.getGridStateRepresentation observation) with hand-written CDNA4 HIP
kernels behind the C-ABI in include/aigar.h, keeping the reference's Python
Model/Field/Player/Cell/Bot surface (see aigar_amd.model / aigar_amd.field).
"""
from . import _abi  # noqa: F401

__all__ = ["_abi"]
