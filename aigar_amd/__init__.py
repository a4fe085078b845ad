"""aigar_amd -- MI355X-native agar.io environment stepper.

Replaces the reference `src/model` hot path (Field.update() tick and
Bot.getGridStateRepresentation observation) with hand-written CDNA4 HIP
kernels behind the C-ABI in include/aigar.h, keeping the reference's Python
Model/Field/Player/Cell/Bot surface.

Modules: `_lib` (ctypes binding, `Stepper`), `model` (the reference's Model /
Field / Player / Cell / Bot / RGBGenerator names over the device), `env`
(batched learner environment), `tiles` (C4: one arena tiled over GPUs),
`replicas` (multi-GPU replica plumbing).
"""
from . import _abi  # noqa: F401

__all__ = ["_abi"]
