"""aigar_run: the whole env step (policy + Field.update + observation) replayed
from one hipGraph must give exactly what the separate calls give -- same world,
same observation rows -- and the graph must be re-captured when its parameters
or its output buffer change."""
import numpy as np
import pytest

from aigar_amd import _abi
from oracle_lib import Oracle, make_config
import parity

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")
_lib = pytest.importorskip("aigar_amd._lib")

CH = (_abi.OBS_PELLET | _abi.OBS_SELF | _abi.OBS_WALL | _abi.OBS_ENEMY | _abi.OBS_VIRUS | _abi.OBS_SELF_SLF
      | _abi.OBS_SELF_LF | _abi.OBS_ENEMY_SLF | _abi.OBS_ENEMY_LF)


def _cfg(bots=96, arenas=1):
    return make_config(n_arenas=arenas, bots=bots, virus=True, max_viruses=24, channels=CH, extras=0x1F)


def _pair(cfg, seed):
    a, b = _lib.Stepper(cfg), _lib.Stepper(cfg)
    for s in (a, b):
        s.set_stream(torch.cuda.current_stream().cuda_stream)
        s.reset(seed)
    return a, b


@pytest.mark.parametrize("policy", ["random", "greedy"])
def test_run_matches_separate_calls(policy):
    cfg = _cfg()
    fused, sep = _pair(cfg, 21)
    oa = torch.zeros((fused.NP, fused.obs_len), dtype=torch.float64, device="cuda")
    ob = torch.zeros_like(oa)
    for t in range(30):
        fused.run(1, policy, oa, p_split=0.05, p_eject=0.05, seed=3, greedy_split=True)
        if policy == "random":
            sep.policy_random(0.05, 0.05, 3)
        else:
            sep.policy_greedy(True)
        sep.step(1)
        sep.observe(ob)
        torch.cuda.synchronize()
        assert torch.equal(torch.nan_to_num(oa, nan=-7.0), torch.nan_to_num(ob, nan=-7.0)), t
    assert parity.diff_states(fused.get_state(), sep.get_state(), ftol=0.0) == []
    fused.close()
    sep.close()


def test_run_multi_step_float32_and_recapture():
    cfg = _cfg(bots=64, arenas=2)
    fused, sep = _pair(cfg, 4)
    o32 = torch.zeros((fused.NP, fused.obs_len), dtype=torch.float32, device="cuda")
    r32 = torch.zeros_like(o32)
    fused.run(5, "random", o32, p_split=0.1, p_eject=0.1, seed=8)  # one 4-step graph replay + one 1-step replay
    for _ in range(5):
        sep.policy_random(0.1, 0.1, 8)
        sep.step(1)
        sep.observe(r32)
    torch.cuda.synchronize()
    assert torch.equal(torch.nan_to_num(o32, nan=-7.0), torch.nan_to_num(r32, nan=-7.0))
    # new parameters and no observation: a new graph, same world as the separate calls
    fused.run(3, "random", None, p_split=0.0, p_eject=0.3, seed=9)
    for _ in range(3):
        sep.policy_random(0.0, 0.3, 9)
        sep.step(1)
    for a in range(2):
        assert parity.diff_states(fused.get_state(a), sep.get_state(a), ftol=0.0) == []
    # policy "none" keeps externally set commands
    cmd = np.random.default_rng(1).uniform(0, 300, (fused.NP, 4))
    cmd[:, 2:] = 0
    fused.set_commands(cmd)
    sep.set_commands(cmd)
    fused.run(2, "none", o32)
    sep.step(1)
    sep.observe(r32)
    sep.step(1)
    sep.observe(r32)
    torch.cuda.synchronize()
    assert torch.equal(torch.nan_to_num(o32, nan=-7.0), torch.nan_to_num(r32, nan=-7.0))
    fused.close()
    sep.close()


@pytest.mark.parametrize("policy", ["random", "greedy"])
def test_unrolled_run_graph_matches_one_step_graph(policy, monkeypatch):
    """aigar_run's multi-step graph (AIGAR_RUN_UNROLL copies of the step in one
    graph, read at aigar_create; default 4) against the one-step graph replayed
    n times: the same world and rows for step counts below, at and past the
    unroll (11 = 8 + 3: one unrolled replay and three one-step replays)."""
    monkeypatch.setenv("AIGAR_RUN_UNROLL", "1")
    one = _lib.Stepper(_cfg(bots=256))
    monkeypatch.setenv("AIGAR_RUN_UNROLL", "8")
    unr = _lib.Stepper(_cfg(bots=256))
    oa = torch.zeros((one.NP, one.obs_len), dtype=torch.float64, device="cuda")
    ob = torch.zeros_like(oa)
    for s in (one, unr):
        s.set_stream(torch.cuda.current_stream().cuda_stream)
        s.reset(31)
    for n in (3, 8, 11):
        one.run(n, policy, oa, p_split=0.05, p_eject=0.05, seed=6, greedy_split=True)
        unr.run(n, policy, ob, p_split=0.05, p_eject=0.05, seed=6, greedy_split=True)
        torch.cuda.synchronize()
        assert torch.equal(torch.nan_to_num(oa, nan=-7.0), torch.nan_to_num(ob, nan=-7.0)), n
        assert parity.diff_states(one.get_state(), unr.get_state(), ftol=0.0) == [], n
    one.close()
    unr.close()


def test_run_rejects_host_buffers_and_bad_policy():
    g = _lib.Stepper(_cfg(bots=8))
    g.reset(1)
    with pytest.raises(ValueError):
        g.run(1, "random", np.zeros((g.NP, g.obs_len)))
    with pytest.raises(KeyError):
        g.run(1, "bogus")
    g.close()


@pytest.mark.parametrize("policy", ["random", "greedy"])
def test_run_many_steps_in_one_call(policy):
    """Many steps in ONE aigar_run call (graph replays back to back): the last
    rows (whose last-frame channels chain through every step's history) and the
    world must equal the separate calls'.  Greedy: inside a call every step's
    observation also makes the next step's Greedy moves (k_observe<..., GR>),
    so steps 2..n take moves the fused observation staged."""
    cfg = _cfg(bots=512)
    fused, sep = _pair(cfg, 12)
    oa = torch.zeros((fused.NP, fused.obs_len), dtype=torch.float64, device="cuda")
    ob = torch.zeros_like(oa)
    for n in (1, 7, 24):
        fused.run(n, policy, oa, p_split=0.05, p_eject=0.05, seed=5, greedy_split=True)
        for _ in range(n):
            if policy == "random":
                sep.policy_random(0.05, 0.05, 5)
            else:
                sep.policy_greedy(True)
            sep.step(1)
            sep.observe(ob)
        torch.cuda.synchronize()
        assert torch.equal(torch.nan_to_num(oa, nan=-7.0), torch.nan_to_num(ob, nan=-7.0)), n
        assert parity.diff_states(fused.get_state(), sep.get_state(), ftol=0.0) == [], n
    fused.close()
    sep.close()


def test_greedy_run_at_c3_matches_separate_calls():
    """The bench's greedy line: the matured C3 world (tick 50), 4096 Greedy bots
    with ENABLE_GREEDY_SPLIT, 40 steps in two aigar_run calls (the fused
    observation stages every move after a call's first) against the policy
    launch + tick + observation as separate calls: rows, world and commands
    identical, with deaths and respawns on the way."""
    import bench
    cfg = bench.make_cfg("c3")
    fused, sep = _lib.Stepper(cfg), _lib.Stepper(cfg)
    for s in (fused, sep):
        s.set_stream(torch.cuda.current_stream().cuda_stream)
        bench.start_world(s, "c3", 1, 1)
    oa = torch.zeros((fused.NP, fused.obs_len), dtype=torch.float64, device="cuda")
    ob = torch.zeros_like(oa)
    for n in (15, 25):
        fused.run(n, "greedy", oa, greedy_split=True)
        for _ in range(n):
            sep.policy_greedy(True)
            sep.step(1)
            sep.observe(ob)
        torch.cuda.synchronize()
        assert torch.equal(torch.nan_to_num(oa, nan=-7.0), torch.nan_to_num(ob, nan=-7.0)), n
        assert parity.diff_states(fused.get_state(), sep.get_state(), ftol=0.0) == [], n
    assert fused.counters()["ticks"] == sep.counters()["ticks"]
    fused.close()
    sep.close()


def _commands(stp):
    st = stp.get_state()
    pf, pi = np.asarray(st["players_f"]), np.asarray(st["players_i"])
    return np.c_[pf[:, 0], pf[:, 1], pi[:, 2], pi[:, 3]].astype(np.float64)


def test_bench_graph_matches_oracle():
    """bench.py's timed path itself -- the C3 workload's config
    (events off, as timed), data/c3_t50.npz loaded by bench.start_world, the aigar_run
    graph with the random policy fused into k_players and the bench's own split /
    eject probabilities and salt -- against the oracle for 25 steps.  The commands
    the fused policy made are read back after every replay and given to the oracle;
    the world and every bot's observation row are compared every step.  A second
    stepper replays the same graph 25 times in ONE call (as the timed region does)
    and must end identical."""
    import bench
    _, _, _, _, ps, pe, _, _, _ = bench.WORKLOADS["c3"]
    salt = 1234  # bench.py --seed default, rank 0
    cfg = bench.make_cfg("c3")
    stp, one = _lib.Stepper(cfg), _lib.Stepper(cfg)
    for s in (stp, one):
        s.set_stream(torch.cuda.current_stream().cuda_stream)
        bench.start_world(s, "c3", salt, 1)
    o = Oracle(cfg)
    o.load_state(parity.load_snapshot("c3_t50"))
    assert parity.diff_states(stp.get_state(), o.get_state(), ftol=0.0) == []
    obs = torch.full((stp.NP, stp.obs_len), -7.0, dtype=torch.float64, device="cuda")
    splits = ejects = 0
    for t in range(25):
        stp.run(1, "random", obs, p_split=ps, p_eject=pe, seed=salt, greedy_split=True)
        torch.cuda.synchronize()
        cmd = _commands(stp)
        splits += int(cmd[:, 2].sum())
        ejects += int(cmd[:, 3].sum())
        o.set_commands(cmd)
        o.step(1)
        want = o.observe()
        dif = parity.diff_states(stp.get_state(), o.get_state())
        assert not dif, "step %d: %s" % (t, dif[:3])
        assert parity.obs_close(obs.cpu().numpy(), want), "step %d: observation rows differ" % t
    assert splits > 0 and ejects > 0, (splits, ejects)
    obs1 = torch.full_like(obs, -7.0)
    one.run(25, "random", obs1, p_split=ps, p_eject=pe, seed=salt, greedy_split=True)
    torch.cuda.synchronize()
    assert torch.equal(torch.nan_to_num(obs1, nan=-7.0), torch.nan_to_num(obs, nan=-7.0))
    assert parity.diff_states(one.get_state(), stp.get_state(), ftol=0.0) == []
    for s in (stp, one, o):
        s.close()
