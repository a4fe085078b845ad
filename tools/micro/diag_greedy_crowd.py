import sys, numpy as np
sys.path[:0] = ['.', 'tests']
from aigar_amd import _abi, _lib
from oracle_lib import Oracle, make_config
cfg = make_config(bots=64, virus=True, max_viruses=30, field_size=250, channels=_abi.OBS_PELLET | _abi.OBS_WALL | _abi.OBS_ENEMY, extras=0x3)
g, o = _lib.Stepper(cfg), Oracle(cfg)
g.reset(4); o.reset(4)
def cmds(st):
    pf, pi = np.asarray(st["players_f"]), np.asarray(st["players_i"])
    return np.c_[pf[:, 0], pf[:, 1], pi[:, 2], pi[:, 3]]
for t in range(400):
    g.policy_greedy(True); o.policy_greedy(True)
    cg, co = cmds(g.get_state()), cmds(o.get_state())
    bad = np.nonzero(np.any(cg != co, axis=1))[0]
    if len(bad):
        sg, so = g.player_stats(), o.player_stats()
        for b in bad:
            print("tick", t, "bot", b, "cmd", cg[b], co[b], "fs", repr(sg[b, 4]), repr(so[b, 4]), "fx", repr(sg[b,2]), repr(so[b,2]), "mass", repr(sg[b,1]), repr(so[b,1]))
        break
    g.step(1); o.step(1)
import parity
sg, so = g.get_state(), o.get_state()
print("diff ftol0:", parity.diff_states(sg, so, ftol=0.0)[:5])
for name, st in (("gpu", sg), ("orc", so)):
    ci, cf = np.asarray(st["cells_i"]), np.asarray(st["cells_f"])
    sel = np.nonzero(ci[:, 0] == 30)[0]
    print(name, "player 30 cells (seq, x, m):", [(int(ci[k, 2]), repr(cf[k, 0]), repr(cf[k, 2])) for k in sel])
