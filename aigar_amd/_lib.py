"""ctypes binding of libaigar_hip.so (include/aigar.h).

There is no CPU fallback: if the HIP library is missing or cannot be loaded
this module raises, so a GPU run can never silently take another path.
"""
import ctypes as C
import os

import numpy as np

from . import _abi

HERE = os.path.dirname(os.path.abspath(__file__))
SO_PATH = os.environ.get("AIGAR_SO") or os.path.join(HERE, "libaigar_hip.so")  # (AIGAR_SO: diagnostics builds)

_lib = None


def _preload_single_hip_runtime():
    """torch ships its own libamdhip64.so (same SONAME as /opt/rocm's).  Two HIP
    runtimes in one process break each other (and make torch streams invalid
    handles for us), so when torch is installed we bind to ITS runtime: preload
    it by path, before our library resolves libamdhip64.so.7.  torch imported
    later resolves to the same file."""
    import importlib.util
    try:
        spec = importlib.util.find_spec("torch")
    except (ImportError, ValueError):
        spec = None
    if spec is None or not spec.submodule_search_locations:
        return None
    cand = os.path.join(list(spec.submodule_search_locations)[0], "lib", "libamdhip64.so")
    if os.path.exists(cand):
        C.CDLL(cand, mode=C.RTLD_GLOBAL)
        return cand
    return None


def rccl_path():
    """The librccl.so this process's torch uses (one HIP runtime for both), else None
    (the loader's librccl.so)."""
    import importlib.util
    spec = importlib.util.find_spec("torch")
    if spec is not None and spec.submodule_search_locations:
        cand = os.path.join(list(spec.submodule_search_locations)[0], "lib", "librccl.so")
        if os.path.exists(cand):
            return cand
    return None


def rccl_unique_id():
    """A fresh ncclUniqueId (128 bytes) for aigar_tile_comm_init (rank 0 makes it)."""
    L = load()
    buf = C.create_string_buffer(128)
    path = rccl_path()
    if L.aigar_rccl_unique_id(path.encode() if path else None, buf) < 0:
        raise RuntimeError("aigar: " + L.aigar_last_error().decode())
    return buf.raw


def load(build_if_missing=False):
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(SO_PATH):
        if build_if_missing:
            from . import _build
            _build.build()
        else:
            raise RuntimeError("libaigar_hip.so not found at %s: build it with `python -m aigar_amd._build` "
                               "(hipcc --offload-arch=gfx950)" % SO_PATH)
    _preload_single_hip_runtime()
    L = C.CDLL(SO_PATH)
    vp, i32, u64, dp = C.c_void_p, C.c_int, C.c_uint64, C.POINTER(C.c_double)
    L.aigar_last_error.restype = C.c_char_p
    L.aigar_abi_version.restype = i32
    sig = {
        "aigar_create": [C.POINTER(_abi.Config), C.POINTER(vp)],
        "aigar_destroy": [vp],
        "aigar_reset": [vp, u64],
        "aigar_set_commands": [vp, vp, i32],
        "aigar_policy_random": [vp, C.c_double, C.c_double, u64],
        "aigar_step": [vp, i32],
        "aigar_obs_len": [vp],
        "aigar_observe": [vp, vp, i32, i32],
        "aigar_observe_pixels": [vp, vp, i32, u64, i32, i32],
        "aigar_set_actions": [vp, vp, vp, i32],
        "aigar_reset_bots": [vp, vp, i32],
        "aigar_player_stats": [vp, vp, i32],
        "aigar_get_state": [vp, i32, C.POINTER(_abi.State)],
        "aigar_load_state": [vp, i32, C.POINTER(_abi.State)],
        "aigar_get_events": [vp, i32, C.POINTER(C.c_int64), i32, C.POINTER(i32)],
        "aigar_set_stream": [vp, vp],
        "aigar_sync": [vp],
        "aigar_profile": [vp, i32],
        "aigar_kernel_time": [vp, C.c_char_p, dp, C.POINTER(i32)],
        "aigar_selftest_pow": [dp, dp, dp, i32],
        "aigar_selftest_trig": [dp, dp, dp, i32],
        "aigar_counters": [vp, i32, C.POINTER(C.c_int64), i32],
        "aigar_policy_greedy": [vp, i32, vp, i32],
        "aigar_apply_actions": [vp, vp, i32, i32, i32, i32, i32],
        "aigar_rewards": [vp, vp, C.POINTER(_abi.RewardParams), i32, i32],
        "aigar_set_split_likelihood": [vp, i32, C.POINTER(C.c_int32)],
        "aigar_run": [vp, i32, C.POINTER(_abi.RunParams), vp, i32],
        "aigar_env_step": [vp, vp, i32, i32, i32, C.POINTER(_abi.RewardParams), vp, vp, i32],
        "aigar_get_events_raw": [vp, i32, C.POINTER(C.c_int64), i32, C.POINTER(i32)],
        "aigar_observe_masked": [vp, vp, i32, i32, vp, i32],
        "aigar_set_roles": [vp, vp, i32],
        "aigar_env_config": [vp, C.POINTER(_abi.EnvParams)],
        "aigar_policy_random_bots": [vp],
        "aigar_tile_info": [vp, C.POINTER(C.c_int32), C.POINTER(vp), C.POINTER(vp), C.POINTER(C.c_int64)],
        "aigar_tile_set_buffers": [vp, vp, vp],
        "aigar_tile_msg_bytes": [vp, C.POINTER(C.c_int64)],
        "aigar_tile_begin": [vp, C.POINTER(_abi.RunParams)],
        "aigar_tile_policy": [vp, i32],
        "aigar_tile_apply_commands": [vp],
        "aigar_tile_apply": [vp, C.POINTER(i32)],
        "aigar_tile_resume": [vp],
        "aigar_tile_end": [vp, vp, i32],
        "aigar_tile_exchange_local": [C.POINTER(vp), i32],
        "aigar_tile_observers": [vp, C.POINTER(C.c_int32)],
        "aigar_rccl_unique_id": [C.c_char_p, vp],
        "aigar_tile_comm_init": [vp, C.c_char_p, vp, i32, i32],
        "aigar_tile_run": [vp, i32, C.POINTER(_abi.RunParams), i32, vp, i32],
        "aigar_tile_run_graphed": [vp],
        "aigar_tile_loopback": [vp],
    }
    for name, args in sig.items():
        f = getattr(L, name, None)
        if f is None and os.environ.get("AIGAR_SO"):  # an older diagnostics build: bind what it has
            continue
        if f is None:
            raise RuntimeError("libaigar_hip.so lacks %s: rebuild it (python -m aigar_amd._build)" % name)
        f.argtypes = args
        f.restype = i32
    if L.aigar_abi_version() != _abi.ABI_VERSION:
        raise RuntimeError("libaigar_hip.so ABI %d != python binding %d" % (L.aigar_abi_version(), _abi.ABI_VERSION))
    _lib = L
    return L


def _ptr(x):
    """Host numpy array or device tensor -> (void pointer, on_device)."""
    if x is None:
        return None, 0
    if isinstance(x, np.ndarray):
        return x.ctypes.data_as(C.c_void_p), 0
    if hasattr(x, "data_ptr"):  # torch tensor (device memory when x.is_cuda)
        return C.c_void_p(x.data_ptr()), int(bool(getattr(x, "is_cuda", False)))
    raise TypeError("expected numpy array or torch tensor, got %r" % type(x))


class Stepper:
    """One handle of the device stepper: n_arenas fields x bots_per_arena players."""

    def __init__(self, cfg):
        self.L = load()
        self.cfg = cfg
        h = C.c_void_p()
        self._chk(self.L.aigar_create(C.byref(cfg), C.byref(h)))
        self.h = h
        self.A, self.B = cfg.n_arenas, cfg.bots_per_arena
        self.NP = self.A * self.B
        self.obs_len = self.L.aigar_obs_len(self.h)

    def _chk(self, r):
        if r < 0:
            raise RuntimeError("aigar: " + self.L.aigar_last_error().decode())
        return r

    def close(self):
        if getattr(self, "_one", None) is not None:
            self._one.close()
            self._one = None
        if getattr(self, "h", None):
            self.L.aigar_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def reset(self, seed=0):
        self._chk(self.L.aigar_reset(self.h, int(seed)))

    def set_commands(self, cmd):
        if isinstance(cmd, np.ndarray):
            cmd = np.ascontiguousarray(cmd, np.float64).reshape(self.NP, 4)
        p, dev = _ptr(cmd)
        self._chk(self.L.aigar_set_commands(self.h, p, dev))

    def policy_random(self, p_split=0.0, p_eject=0.0, seed=0):
        self._chk(self.L.aigar_policy_random(self.h, float(p_split), float(p_eject), int(seed)))

    def policy_greedy(self, greedy_split=False, mask=None):
        """Greedy bots' moves (bot.py:579-633) for the players where mask != 0 (all if None)."""
        if isinstance(mask, np.ndarray):
            mask = np.ascontiguousarray(mask, np.uint8).reshape(self.NP)
        p, dev = _ptr(mask)
        self._chk(self.L.aigar_policy_greedy(self.h, int(bool(greedy_split)), p, dev))

    def apply_actions(self, act, enable_split=True, skipping=False, record=True):
        """Learner actions act[NP, n] (n = 2..4, numpy or device tensor) through set_command_point."""
        if isinstance(act, np.ndarray):
            act = np.ascontiguousarray(act, np.float64).reshape(self.NP, -1)
        n = int(act.shape[1])
        p, dev = _ptr(act)
        self._chk(self.L.aigar_apply_actions(self.h, p, n, int(bool(enable_split)), int(bool(skipping)),
                                             int(bool(record)), dev))

    def rewards(self, params=None, update_last=True, out=None):
        """Bot.getReward for every player (NaN where the reference has None)."""
        prm = params if isinstance(params, _abi.RewardParams) else _abi.RewardParams.from_parameters(params)
        if out is None:
            out = np.zeros(self.NP, np.float64)
        p, dev = _ptr(out)
        self._chk(self.L.aigar_rewards(self.h, p, C.byref(prm), int(bool(update_last)), dev))
        return out

    def set_split_likelihood(self, lh, arena=0):
        if lh is None:
            self._chk(self.L.aigar_set_split_likelihood(self.h, arena, None))
            return
        a = np.ascontiguousarray(lh, np.int32).reshape(self.B)
        self._chk(self.L.aigar_set_split_likelihood(self.h, arena, a.ctypes.data_as(C.POINTER(C.c_int32))))

    def step(self, n=1):
        self._chk(self.L.aigar_step(self.h, int(n)))

    def run(self, n, policy="random", out=None, p_split=0.0, p_eject=0.0, seed=0, greedy_split=False):
        """n whole env steps (policy + Field.update + observation into the DEVICE tensor out,
        or no observation when out is None), replayed from one captured hipGraph."""
        pol = {"none": _abi.POLICY_NONE, "random": _abi.POLICY_RANDOM, "greedy": _abi.POLICY_GREEDY}[policy]
        prm = _abi.RunParams(pol, int(bool(greedy_split)), float(p_split), float(p_eject), int(seed))
        p, dt = None, 0
        if out is not None:
            if not getattr(out, "is_cuda", False):
                raise ValueError("aigar_run writes observations to a device tensor")
            dt = 0 if str(out.dtype) == "torch.float64" else 1
            if tuple(out.shape) != (self.NP, self.obs_len):
                raise ValueError("observation tensor must be [%d, %d]" % (self.NP, self.obs_len))
            p = C.c_void_p(out.data_ptr())
        self._chk(self.L.aigar_run(self.h, int(n), C.byref(prm), p, dt))
        return out

    def env_step(self, act, reward, obs, enable_split=True, skip=0, params=None):
        """One learner decision on device tensors (aigar_env_step): act [NP, 2..4] float64,
        reward [NP] float64 (summed over the skip + 1 ticks), obs [NP, obs_len]; one graph replay."""
        for t in (act, reward, obs):
            if not getattr(t, "is_cuda", False) or not t.is_contiguous():
                raise ValueError("env_step takes contiguous device tensors")
        if str(act.dtype) != "torch.float64" or str(reward.dtype) != "torch.float64":
            raise ValueError("actions and rewards are float64")
        if act.dim() != 2 or act.shape[0] != self.NP or not 2 <= act.shape[1] <= 4:
            raise ValueError("actions must be [%d, 2..4]" % self.NP)
        if tuple(obs.shape) != (self.NP, self.obs_len) or tuple(reward.shape) != (self.NP,):
            raise ValueError("reward must be [%d], obs [%d, %d]" % (self.NP, self.NP, self.obs_len))
        prm = params if isinstance(params, _abi.RewardParams) else _abi.RewardParams.from_parameters(params)
        dt = 0 if str(obs.dtype) == "torch.float64" else 1
        self._chk(self.L.aigar_env_step(self.h, C.c_void_p(act.data_ptr()), int(act.shape[1]), int(bool(enable_split)),
                                        int(skip), C.byref(prm), C.c_void_p(reward.data_ptr()),
                                        C.c_void_p(obs.data_ptr()), dt))

    def _check_out(self, out, shape, dtypes, what):
        """The library writes prod(shape) elements of the dtype into out: refuse a
        buffer of another shape / dtype, a strided view or a tensor on another device."""
        d = str(getattr(out, "dtype", "")).replace("torch.", "")
        if tuple(out.shape) != tuple(shape):
            raise ValueError("%s: out must have shape %s, got %s" % (what, tuple(shape), tuple(out.shape)))
        if d not in dtypes:
            raise ValueError("%s: out dtype must be one of %s, got %s" % (what, dtypes, d))
        contig = out.flags["C_CONTIGUOUS"] if isinstance(out, np.ndarray) else out.is_contiguous()
        if not contig:
            raise ValueError("%s: out must be C-contiguous" % what)
        if hasattr(out, "is_cuda") and out.is_cuda and out.device.index not in (None, self.cfg.device):
            raise ValueError("%s: out is on cuda:%s, the stepper on device %d" % (what, out.device.index,
                                                                                 self.cfg.device))
        return d

    def observe(self, out=None, dtype=np.float64, mask=None):
        """getStateRepresentation of every player (mask: only where mask != 0; the
        other rows of out are kept and those bots' history does not advance)."""
        if out is None:
            out = np.zeros((self.NP, self.obs_len), dtype)
        d = self._check_out(out, (self.NP, self.obs_len), ("float64", "float32"), "observe")
        dt = 0 if d == "float64" else 1
        p, dev = _ptr(out)
        if mask is None:
            self._chk(self.L.aigar_observe(self.h, p, dt, dev))
        else:
            if isinstance(mask, np.ndarray):
                mask = np.ascontiguousarray(mask, np.uint8).reshape(self.NP)
            mp, mdev = _ptr(mask)
            self._chk(self.L.aigar_observe_masked(self.h, p, dt, dev, mp, mdev))
        return out

    def set_roles(self, roles):
        """Player roles of a mixed population: AIGAR_ROLE_* codes or "NN" / "Greedy" / "Random"."""
        r = np.array([_abi.ROLES.get(x, x) if isinstance(x, str) else x for x in roles], np.uint8).reshape(self.NP)
        self._chk(self.L.aigar_set_roles(self.h, r.ctypes.data_as(C.c_void_p), 0))

    def env_config(self, greedy_split=False, random_skip=7, random_split=False, random_eject=False, salt=0):
        prm = _abi.EnvParams(int(bool(greedy_split)), int(random_skip), int(bool(random_split)),
                             int(bool(random_eject)), int(salt))
        self._chk(self.L.aigar_env_config(self.h, C.byref(prm)))

    def policy_random_bots(self):
        self._chk(self.L.aigar_policy_random_bots(self.h))

    def reset_arena(self, arena, seed):
        """Field.reset of ONE arena of a batched handle (a fresh world keyed by seed;
        that arena's bots reset as by load_state), the others untouched."""
        if self.A == 1:
            return self.reset(seed)
        c = _abi.Config()
        C.memmove(C.byref(c), C.byref(self.cfg), C.sizeof(_abi.Config))
        c.n_arenas = 1
        if getattr(self, "_one", None) is None:
            self._one = Stepper(c)
        self._one.reset(seed)
        self.load_state(self._one.get_state(0), arena)

    def observe_pixels(self, side=42, color_seed=0, rgb=True, out=None):
        """RGBGenerator.get_cnn_inputRGB for every player (rgbGenerator.py:95-110):
        uint8 [NP, side, side, 3] when rgb, else float64/float32 grayscale [NP, side, side]."""
        if out is None:
            out = np.zeros((self.NP, side, side, 3), np.uint8) if rgb else np.zeros((self.NP, side, side), np.float64)
        d = str(getattr(out, "dtype", "")).replace("torch.", "")
        if d == "uint8":
            self._check_out(out, (self.NP, side, side, 3), ("uint8",), "observe_pixels")
        else:
            self._check_out(out, (self.NP, side, side), ("float64", "float32"), "observe_pixels")
        dt = 2 if d == "uint8" else 0 if d == "float64" else 1
        p, dev = _ptr(out)
        self._chk(self.L.aigar_observe_pixels(self.h, p, int(side), int(color_seed), dt, dev))
        return out

    def set_actions(self, cur=None, prev=None):
        c = None if cur is None else np.ascontiguousarray(cur, np.float64)
        q = None if prev is None else np.ascontiguousarray(prev, np.float64)
        self._chk(self.L.aigar_set_actions(self.h, _ptr(c)[0], _ptr(q)[0], 0))

    def reset_bots(self, mask=None):
        """Bot.reset's device half (bot.py:125-164) for the players where mask != 0
        (all if None): history grids zeroed, lastFovSize 0."""
        if isinstance(mask, np.ndarray):
            mask = np.ascontiguousarray(mask, np.uint8).reshape(self.NP)
        p, dev = _ptr(mask)
        self._chk(self.L.aigar_reset_bots(self.h, p, dev))

    def player_stats(self):
        out = np.zeros((self.NP, 5), np.float64)
        self._chk(self.L.aigar_player_stats(self.h, out.ctypes.data_as(C.c_void_p), 0))
        return out

    def get_state(self, arena=0):
        cnt = _abi.State()
        self._chk(self.L.aigar_get_state(self.h, arena, C.byref(cnt)))
        st, arrays = _abi.alloc_state(cnt)
        self._chk(self.L.aigar_get_state(self.h, arena, C.byref(st)))
        return _abi.struct_to_dict(st, arrays)

    def load_state(self, d, arena=0):
        st, keep = _abi.state_to_struct(d)
        self._chk(self.L.aigar_load_state(self.h, arena, C.byref(st)))

    def events(self, arena=0):
        n = C.c_int(0)
        self._chk(self.L.aigar_get_events(self.h, arena, None, 0, C.byref(n)))
        out = np.zeros((n.value, 4), np.int64)
        if n.value:
            self._chk(self.L.aigar_get_events(self.h, arena, out.ctypes.data_as(C.POINTER(C.c_int64)), n.value,
                                              C.byref(n)))
        return out

    def events_raw(self, arena=0):
        """Unsorted event rows with their sort keys: (key_hi, key_lo, code, a, b)."""
        n = C.c_int(0)
        self._chk(self.L.aigar_get_events_raw(self.h, arena, None, 0, C.byref(n)))
        out = np.zeros((n.value, 5), np.int64)
        if n.value:
            self._chk(self.L.aigar_get_events_raw(self.h, arena, out.ctypes.data_as(C.POINTER(C.c_int64)), n.value,
                                                  C.byref(n)))
        return out

    # ---- C4 tiles (include/aigar.h: aigar_tile_*)
    def tile_info(self):
        info = (C.c_int32 * 14)()
        ob, ib, nb = C.c_void_p(), C.c_void_p(), C.c_int64(0)
        self._chk(self.L.aigar_tile_info(self.h, info, C.byref(ob), C.byref(ib), C.byref(nb)))
        v = list(info)
        return {"ntiles": v[0], "tile_id": v[1], "own": tuple(v[2:6]), "held": tuple(v[6:10]), "tcap": v[10],
                "bm_words": v[11], "hcap": v[12], "hrec": v[13], "handoff_bytes": v[12] * v[13] * 32,
                "outbox": ob.value, "inbox": ib.value, "msg_bytes": nb.value}

    def tile_msg_bytes(self):
        """Bytes of the current pass's message (the first pass sends no bitmap)."""
        n = C.c_int64(0)
        self._chk(self.L.aigar_tile_msg_bytes(self.h, C.byref(n)))
        return n.value

    def tile_set_buffers(self, outbox_ptr, inbox_ptr):
        self._chk(self.L.aigar_tile_set_buffers(self.h, C.c_void_p(int(outbox_ptr)), C.c_void_p(int(inbox_ptr))))

    def tile_begin(self, policy="none", p_split=0.0, p_eject=0.0, seed=0):
        """policy "greedy": this tick's commands must have gone round already
        (tile_policy, the exchange, tile_apply_commands)."""
        pol = {"none": _abi.POLICY_NONE, "random": _abi.POLICY_RANDOM, "greedy": _abi.POLICY_GREEDY}[policy]
        prm = _abi.RunParams(pol, 0, float(p_split), float(p_eject), int(seed))
        self._chk(self.L.aigar_tile_begin(self.h, C.byref(prm)))

    def tile_policy(self, greedy_split=False):
        """Greedy moves (bot.py:579-633) of the bots this tile observes, into the
        command message the transport all-gathers next."""
        self._chk(self.L.aigar_tile_policy(self.h, 1 if greedy_split else 0))

    def tile_apply_commands(self):
        """The other tiles' Greedy commands (after the exchange of tile_policy's messages)."""
        self._chk(self.L.aigar_tile_apply_commands(self.h))

    def tile_apply(self, wait=True):
        """Apply the gathered messages; wait: return the owned cells still undone on
        all tiles (a host round trip), else None (the next pass gates itself)."""
        if not wait:
            self._chk(self.L.aigar_tile_apply(self.h, None))
            return None
        u = C.c_int(0)
        self._chk(self.L.aigar_tile_apply(self.h, C.byref(u)))
        return u.value

    def tile_observers(self):
        """Per player: the tile that computed its row at the last observation (-1: dead)."""
        out = np.zeros(self.NP, np.int32)
        self._chk(self.L.aigar_tile_observers(self.h, out.ctypes.data_as(C.POINTER(C.c_int32))))
        return out

    def tile_resume(self):
        self._chk(self.L.aigar_tile_resume(self.h))

    def tile_comm_init(self, uid, nranks, rank):
        """This tile's RCCL communicator (ncclCommInitRank): nranks = tiles, rank = tile id."""
        path = rccl_path()
        buf = C.create_string_buffer(bytes(uid), 128)
        self._chk(self.L.aigar_tile_comm_init(self.h, path.encode() if path else None, buf, int(nranks), int(rank)))

    def tile_run(self, n=1, policy="random", out=None, p_split=0.0, p_eject=0.0, seed=0, extra_passes=0,
                 greedy_split=False):
        """n tiled steps over RCCL (aigar_tile_run): policy (greedy: each tile moves the bots
        it observes, the commands all-gathered first) + the tick with its all-gathered eat
        passes + the observation of this tile's bots into the DEVICE tensor out."""
        pol = {"none": _abi.POLICY_NONE, "random": _abi.POLICY_RANDOM, "greedy": _abi.POLICY_GREEDY}[policy]
        prm = _abi.RunParams(pol, 1 if greedy_split else 0, float(p_split), float(p_eject), int(seed))
        p, dt = None, 0
        if out is not None:
            if not getattr(out, "is_cuda", False) or tuple(out.shape) != (self.NP, self.obs_len):
                raise ValueError("tile_run writes observations to a device tensor [%d, %d]" % (self.NP, self.obs_len))
            dt = 0 if str(out.dtype) == "torch.float64" else 1
            p = C.c_void_p(out.data_ptr())
        self._chk(self.L.aigar_tile_run(self.h, int(n), C.byref(prm), int(extra_passes), p, dt))

    def tile_run_graphed(self):
        return bool(self.L.aigar_tile_run_graphed(self.h))

    def tile_loopback(self):
        """Timing rehearsal (include/aigar.h aigar_tile_loopback): tile_run without a
        communicator, every other tile's message empty."""
        self._chk(self.L.aigar_tile_loopback(self.h))

    def tile_end(self, out=None):
        p, dt = None, 0
        if out is not None:
            if not getattr(out, "is_cuda", False) or tuple(out.shape) != (self.NP, self.obs_len):
                raise ValueError("tile_end writes observations to a device tensor [%d, %d]" % (self.NP, self.obs_len))
            dt = 0 if str(out.dtype) == "torch.float64" else 1
            p = C.c_void_p(out.data_ptr())
        self._chk(self.L.aigar_tile_end(self.h, p, dt))

    COUNTERS = ("vb_serial", "pv_serial", "food_serial", "pellets_eaten", "pp_serial_players", "pellets_spawned",
                "pp_parallel_ticks",
                "ticks")

    def counters(self, arena=0):
        out = np.zeros(8, np.int64)
        self._chk(self.L.aigar_counters(self.h, arena, out.ctypes.data_as(C.POINTER(C.c_int64)), 8))
        return {k: int(v) for k, v in zip(self.COUNTERS, out) if k != "-"}

    def set_stream(self, stream_ptr):
        self._chk(self.L.aigar_set_stream(self.h, C.c_void_p(int(stream_ptr))))

    def sync(self):
        self._chk(self.L.aigar_sync(self.h))

    def profile(self, enable=True):
        self._chk(self.L.aigar_profile(self.h, int(bool(enable))))

    def kernel_time(self, name):
        ms, n = C.c_double(0), C.c_int(0)
        self._chk(self.L.aigar_kernel_time(self.h, name.encode(), C.byref(ms), C.byref(n)))
        return ms.value, n.value


def tile_exchange_local(steppers):
    """In-process transport of a tiled arena: every tile's outbox into every tile's inbox."""
    L = load()
    arr = (C.c_void_p * len(steppers))(*[s.h.value for s in steppers])
    if L.aigar_tile_exchange_local(arr, len(steppers)) < 0:
        raise RuntimeError("aigar: " + L.aigar_last_error().decode())


def selftest_trig(y, x):
    """Device atan2(y, x), sin(x), cos(x) (glibc's, restated in aigar_glibc_trig.h) for host arrays."""
    L = load()
    x = np.ascontiguousarray(x, np.float64)
    y = np.ascontiguousarray(y, np.float64)
    out = np.zeros(3 * len(x))
    dp = C.POINTER(C.c_double)
    if L.aigar_selftest_trig(y.ctypes.data_as(dp), x.ctypes.data_as(dp), out.ctypes.data_as(dp), len(x)) < 0:
        raise RuntimeError("aigar: " + L.aigar_last_error().decode())
    n = len(x)
    return out[:n], out[n:2 * n], out[2 * n:]


def selftest_pow(x, y):
    """Device pow (glibc's, restated in aigar_math.h) for host arrays (diagnostics)."""
    L = load()
    x = np.ascontiguousarray(x, np.float64)
    y = np.ascontiguousarray(y, np.float64)
    out = np.zeros_like(x)
    dp = C.POINTER(C.c_double)
    if L.aigar_selftest_pow(x.ctypes.data_as(dp), y.ctypes.data_as(dp), out.ctypes.data_as(dp), len(x)) < 0:
        raise RuntimeError("aigar: " + L.aigar_last_error().decode())
    return out
