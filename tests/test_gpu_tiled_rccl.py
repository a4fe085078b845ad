"""GPU: the C4 exchange over RCCL on the one GPU of the test box.

The production C4 path (bench.py on the nccl backend) steps each rank's tile
with `aigar_tile_run`: the tick, its eat passes with the exchange as an
ncclAllGather on the tile's stream, and the observation -- one captured
hipGraph per step.  One GPU cannot hold two RCCL ranks, so the test runs the
whole field as ONE forced tile (AIGAR_TILE_FORCE: every tile pass, message,
hand-off plan and apply still runs) over a 1-rank communicator, and checks the
result against the untiled oracle: events every tick, the state, and every
bot's observation.  The same forced tile is also driven through
`TorchTransport(staged=False)` in a world-size-1 `nccl` process group (RCCL
through torch.distributed, in place on torch's stream)."""
import os
import socket

import numpy as np
import pytest

from aigar_amd import _abi
from oracle_lib import Oracle, make_config
import parity

pytestmark = pytest.mark.gpu
_lib = pytest.importorskip("aigar_amd._lib")
torch = pytest.importorskip("torch")
from aigar_amd import tiles  # noqa: E402

C3_CH = (_abi.OBS_PELLET | _abi.OBS_SELF | _abi.OBS_WALL | _abi.OBS_ENEMY | _abi.OBS_VIRUS | _abi.OBS_SELF_LF
         | _abi.OBS_ENEMY_LF)


def c3_config():
    return make_config(bots=4096, field_size=4800, virus=True, max_pellets=100000.0, channels=C3_CH, extras=0x1F,
                       flags=_abi.FLAG_EVENTS)


def forced_tile(cfg):
    return _lib.Stepper(tiles.tile_config(cfg, 1, 1, 0, cap=4096, flags=_abi.TILE_FORCE))


def _policy_commands(stp):
    st = stp.get_state()
    pf, pi = np.asarray(st["players_f"]), np.asarray(st["players_i"])
    return np.c_[pf[:, 0], pf[:, 1], pi[:, 2], pi[:, 3]].astype(np.float64)


@pytest.mark.parametrize("extra", [0, 1])
def test_tile_run_over_rccl_matches_oracle(extra):
    """aigar_tile_run with a 1-rank RCCL communicator, from the matured C3 world:
    the device's random policy (its commands are read back and given to the
    oracle), 30 graph-replayed steps with the observation, then 5 profiled steps
    (direct launches); extra=1 adds the gated second pass with its all-gather."""
    cfg = c3_config()
    stp, o = forced_tile(cfg), Oracle(cfg)
    snap = parity.load_snapshot("c3_t600")
    stp.load_state(snap)
    o.load_state(snap)
    torch.cuda.set_device(0)
    stp.set_stream(torch.cuda.current_stream().cuda_stream)
    tiles.rccl_comm(stp)
    obs = torch.full((cfg.bots_per_arena, stp.obs_len), -7.0, dtype=torch.float64, device="cuda")
    for t in range(35):
        if t == 30:
            stp.profile(True)
        stp.tile_run(1, "random", obs, p_split=2.5e-3, p_eject=1e-2, seed=77, extra_passes=extra)
        torch.cuda.synchronize()
        if t == 0:
            graphed = stp.tile_run_graphed()
        o.set_commands(_policy_commands(stp))
        o.step(1)
        assert np.array_equal(tiles.merge_events([stp.events_raw()]), o.events()), "tick %d: events differ" % t
        want = o.observe()  # (every tick: the last-frame channels carry the previous observation)
        if t % 10 == 9 or t == 34:
            dif = parity.diff_states(stp.get_state(), o.get_state())
            assert not dif, "tick %d: %s" % (t, dif[:3])
            assert parity.obs_close(obs.cpu().numpy(), want), "tick %d: observations differ" % t
    ms, n = stp.kernel_time("exchange")
    assert n == 5 * (1 + extra), (ms, n)
    stp.profile(False)
    stp.sync()
    print("tile_run graphed:", graphed, "exchange ms/launch %.4f" % (ms / n))
    assert graphed, "the RCCL all-gather was not captured into the step's graph"
    stp.close()
    o.close()


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def test_torch_transport_nccl_world_size_one():
    """The TorchTransport path (torch.distributed all_gather_into_tensor, in place
    on torch's stream) over a real `nccl` (RCCL) process group of one rank."""
    import torch.distributed as dist
    cfg = make_config(bots=512, field_size=1700, virus=True, max_viruses=40, channels=C3_CH, extras=0x1F,
                      flags=_abi.FLAG_EVENTS)
    torch.cuda.set_device(0)
    dist.init_process_group("nccl", init_method="tcp://127.0.0.1:%d" % _free_port(), rank=0, world_size=1)
    try:
        stp, o = forced_tile(cfg), Oracle(cfg)
        stp.reset(21)
        o.reset(21)
        tr = tiles.TorchTransport.for_stepper(stp, staged=False)
        obs = torch.empty((512, stp.obs_len), dtype=torch.float64, device="cuda")
        rng = np.random.default_rng(21)
        for t in range(40):
            cmd = parity.synthetic_commands(rng, None, 512, 1700, 0.02, 0.05)
            stp.set_commands(cmd)
            o.set_commands(cmd)
            tiles.tiled_tick([stp], tr, obs=[obs], extra_passes=0)
            o.step(1)
            assert np.array_equal(tiles.merge_events([stp.events_raw()]), o.events()), "tick %d" % t
            want = o.observe()  # (every tick, as the device: the last-frame channels carry the previous one)
        torch.cuda.synchronize()
        dif = parity.diff_states(stp.get_state(), o.get_state())
        assert not dif, dif
        assert parity.obs_close(obs.cpu().numpy(), want)
        assert tr.avg_exchange_ms() is not None
        stp.close()
        o.close()
    finally:
        dist.destroy_process_group()


def test_tile_run_greedy_over_rccl_matches_oracle():
    """aigar_tile_run with policy GREEDY over the 1-rank RCCL communicator: the
    tile moves the bots it observes, the command message goes through its own
    ncclAllGather inside the step graph before the tick; 20 steps from the
    matured tick-50 world, every command equal to the oracle's Greedy move."""
    cfg = c3_config()
    stp, o = forced_tile(cfg), Oracle(cfg)
    snap = parity.load_snapshot("c3_t50")
    stp.load_state(snap)
    o.load_state(snap)
    torch.cuda.set_device(0)
    stp.set_stream(torch.cuda.current_stream().cuda_stream)
    tiles.rccl_comm(stp)
    obs = torch.full((cfg.bots_per_arena, stp.obs_len), -7.0, dtype=torch.float64, device="cuda")
    for t in range(20):
        o.policy_greedy(True)
        want = o.commands()
        stp.tile_run(1, "greedy", obs, greedy_split=True)
        torch.cuda.synchronize()
        got = _policy_commands(stp)
        bad = np.argwhere(got != want)
        assert not len(bad), "step %d bot %d: %s vs oracle %s" % (t, bad[0][0], got[bad[0][0]], want[bad[0][0]])
        o.step(1)
        assert np.array_equal(tiles.merge_events([stp.events_raw()]), o.events()), "step %d: events differ" % t
        want_obs = o.observe()
        if t % 5 == 4:
            dif = parity.diff_states(stp.get_state(), o.get_state())
            assert not dif, "step %d: %s" % (t, dif[:3])
            assert parity.obs_close(obs.cpu().numpy(), want_obs), "step %d: observations differ" % t
    assert stp.tile_run_graphed()
    stp.sync()
