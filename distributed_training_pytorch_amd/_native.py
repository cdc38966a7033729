"""ctypes binding of ``_lib/libdtp.so`` (the HIP/CDNA4 kernels + native runtime).

The library has a plain C ABI (``csrc/dtp_api.h``); the ``ctypes.Structure``
mirrors below must match it field for field.

Policy: on a machine with a GPU the native path is REQUIRED — every op that has
a HIP kernel raises ``NativeUnavailable`` instead of silently falling back to
PyTorch when the library is missing.  CPU tensors (the gloo test paths) use the
PyTorch reference implementations in ``ops/``.
"""
from __future__ import annotations

import ctypes
import os
import threading
from pathlib import Path

import torch  # noqa: F401  -- must be imported first: libdtp.so binds to torch's HIP runtime

# DTP_LIB selects an A/B build (``build.variant``); default: the in-tree library
LIB_PATH = Path(os.environ.get("DTP_LIB") or Path(__file__).resolve().parent / "_lib" / "libdtp.so")

c_int = ctypes.c_int
c_float = ctypes.c_float
c_double = ctypes.c_double
c_void_p = ctypes.c_void_p
c_size_t = ctypes.c_size_t
c_longlong = ctypes.c_longlong
c_uint64 = ctypes.c_uint64


class NativeUnavailable(RuntimeError):
    pass


class SamplerCfg(ctypes.Structure):
    _fields_ = [
        ("mode", c_int),
        ("n", c_int),
        ("world", c_int),
        ("rank", c_int),
        ("batch", c_int),
        ("num_samples", c_int),
        ("steps_per_epoch", c_int),
        ("bits", c_int),
        ("seed", c_uint64),
        ("perm", c_void_p),
        ("perm_epochs", c_int),
        ("pad_", c_int),
    ]


class Hyper(ctypes.Structure):
    _fields_ = [
        ("lr", c_double),
        ("beta1", c_double),
        ("beta2", c_double),
        ("eps", c_double),
        ("weight_decay", c_double),
        ("momentum", c_double),
        ("slope", c_float),
        ("grad_scale", c_float),
    ]


class TrainArgs(ctypes.Structure):
    _fields_ = [
        ("X", c_void_p),
        ("Y", c_void_p),
        ("idx", c_void_p),
        ("params", c_void_p),
        ("opt_m", c_void_p),
        ("opt_v", c_void_p),
        ("step", c_void_p),
        ("grad_out", c_void_p),
        ("loss_log", c_void_p),
        ("status", c_void_p),
        ("peers", c_void_p),
        ("epoch", c_void_p),
        ("wsp", c_void_p),
        ("loss_log_cap", c_int),
        ("n_models", c_int),
        ("n_steps", c_int),
        ("loss", c_int),
        ("cache_data", c_int),
        ("timeout_us", c_int),
        ("bf16", c_int),
        ("host_t0", c_int),
        ("smp", SamplerCfg),
        ("hp", Hyper),
        ("adam_tab", c_void_p),
        ("adam_tab_len", c_int),
        ("xbuf_bytes", c_int),
        ("grp_buf", c_void_p),
        ("grp_epoch", c_void_p),
        ("grp_status", c_void_p),
        ("groups", c_int),
        ("pad3_", c_int),
    ]


class StageArgs(ctypes.Structure):
    _fields_ = [
        ("x", c_void_p),
        ("params", c_void_p),
        ("out", c_void_p),
        ("saved", c_void_p),
        ("grad_out", c_void_p),
        ("grad_in", c_void_p),
        ("grad_params", c_void_p),
        ("out_peer", c_void_p),
        ("batch", c_int),
        ("slope", c_float),
        ("accumulate", c_int),
        ("bf16", c_int),
    ]


STAGE_MULTI_MAX = 4


class StageMulti(ctypes.Structure):
    _fields_ = [
        ("stage", StageArgs * STAGE_MULTI_MAX),
        ("n", c_int),
        ("pad_", c_int),
    ]


class SplitStageArgs(ctypes.Structure):
    _fields_ = [
        ("X", c_void_p),
        ("Y", c_void_p),
        ("params", c_void_p),
        ("opt_m", c_void_p),
        ("opt_v", c_void_p),
        ("step", c_void_p),
        ("loss_log", c_void_p),
        ("status", c_void_p),
        ("act_in", c_void_p),
        ("act_out", c_void_p),
        ("grad_in", c_void_p),
        ("grad_out", c_void_p),
        ("dp_peers", c_void_p),
        ("loss_log_cap", c_int),
        ("n_steps", c_int),
        ("timeout_us", c_int),
        ("cache_data", c_int),
        ("dp_world", c_int),
        ("dp_rank", c_int),
        ("optim", c_int),
        ("link_local", c_int),
        ("smp", SamplerCfg),
        ("hp", Hyper),
        ("grp_buf", c_void_p),
    ]


SPLIT_MAX_LOCAL = 8


class SplitLaunch(ctypes.Structure):
    _fields_ = [
        ("stage", SplitStageArgs * SPLIT_MAX_LOCAL),
        ("shape_id", c_int * SPLIT_MAX_LOCAL),
        ("n", c_int),
        ("members", c_int),
    ]


class OptArgs(ctypes.Structure):
    _fields_ = [
        ("params", c_void_p),
        ("opt_m", c_void_p),
        ("opt_v", c_void_p),
        ("step", c_void_p),
        ("grad", c_void_p),
        ("loss_log", c_void_p),
        ("loss_log_cap", c_int),
        ("n_models", c_int),
        ("P", c_int),
        ("kind", c_int),
        ("loss_scale", c_float),
        ("flags", c_int),
        ("hp", Hyper),
        ("shadow", c_void_p),
        ("shadow_ld", c_longlong),
    ]


class GemmArgs(ctypes.Structure):
    _fields_ = [
        ("A", c_void_p),
        ("B", c_void_p),
        ("C", c_void_p),
        ("bias", c_void_p),
        ("aux", c_void_p),
        ("lda", c_longlong),
        ("ldb", c_longlong),
        ("ldc", c_longlong),
        ("ldaux", c_longlong),
        ("M", c_int),
        ("N", c_int),
        ("K", c_int),
        ("dtype", c_int),
        ("out_dtype", c_int),
        ("trans_a", c_int),
        ("trans_b", c_int),
        ("act", c_int),
        ("accumulate", c_int),
        ("splitk", c_int),
        ("alpha", c_float),
        ("slope", c_float),
        ("vec_a", c_int),
        ("vec_b", c_int),
        ("force_big", c_int),
        ("fast", c_int),
        ("pad_", c_int),
        ("work", c_void_p),
        ("work_bytes", c_longlong),
    ]


DT_F32, DT_BF16 = 0, 1
MODE_GRAD, MODE_ADAM, MODE_SGD, MODE_XGMI_ADAM, MODE_XGMI_SGD = 0, 1, 2, 3, 4
LOSS_MSE, LOSS_CE = 0, 1
SAMPLER_EXPLICIT, SAMPLER_DIST_SHUFFLE, SAMPLER_SEQUENTIAL, SAMPLER_DIST_NOSHUFFLE, SAMPLER_TABLE = 0, 1, 2, 3, 4

_lib = None
_lock = threading.Lock()


def _declare(lib):
    P = ctypes.POINTER
    sig = {
        "dtp_version": (c_int, []),
        "dtp_source_hash": (ctypes.c_char_p, []),
        "dtp_last_error": (ctypes.c_char_p, []),
        "dtp_runtime_last_error": (ctypes.c_char_p, []),
        "dtp_mlp_supported": (c_int, [c_int] * 5),
        "dtp_mlp_supported_bf16": (c_int, [c_int] * 5),
        "dtp_mlp_param_count": (c_int, [c_int] * 4),
        "dtp_mlp_workspace_floats": (c_int, [c_int] * 4),
        "dtp_mlp_train_bf16_supported": (c_int, [c_int] * 4),
        "dtp_mlp_train": (c_int, [P(TrainArgs), c_int, c_int, c_int, c_int, c_int, c_void_p]),
        "dtp_mlp_train_profile": (c_int, [P(TrainArgs), c_void_p]),
        "dtp_xgmi_fused_buffer_bytes": (c_longlong, [c_int, c_int, c_int]),
        "dtp_train_engine_create": (c_void_p, [P(TrainArgs), c_int, c_int, c_int, c_int, c_int]),
        "dtp_train_engine_poison": (c_int, [c_void_p, c_int]),
        "dtp_train_engine_run": (c_int, [c_void_p, c_int, c_int, c_void_p]),
        "dtp_train_engine_destroy": (None, [c_void_p]),
        "dtp_train_engine_lanes": (c_int, [c_void_p]),
        "dtp_train_engine_groups": (c_int, [c_void_p]),
        "dtp_train_engine_profile": (c_int, [c_void_p, c_int, c_int, c_void_p, c_void_p]),
        "dtp_train_engine_status": (c_int, [c_void_p, P(c_int)]),
        "dtp_mlp_train_lanes": (c_int, [P(TrainArgs), c_int, c_int, c_int, c_int, c_int]),
        "dtp_mlp_train_profile_lanes": (c_int, [P(TrainArgs), c_int, c_void_p]),
        "dtp_mlp_stage_fwd": (c_int, [P(StageArgs), c_int, c_int, c_int, c_int, c_int, c_void_p]),
        "dtp_mlp_stage_fwd_multi": (c_int, [P(StageMulti), c_int, c_int, c_int, c_int, c_int, c_void_p]),
        "dtp_mlp_stage_bwd": (c_int, [P(StageArgs), c_int, c_int, c_int, c_int, c_int, c_void_p]),
        "dtp_flat_optimizer": (c_int, [P(OptArgs), c_void_p]),
        "dtp_mlp_stage_bwd_opt": (c_int, [P(StageMulti), P(OptArgs), c_int, c_int, c_int, c_int, c_int, c_void_p]),
        "dtp_mse_max_elems": (c_longlong, []),
        "dtp_mse_fwd": (c_int, [c_void_p, c_void_p, c_longlong, c_void_p, c_void_p]),
        "dtp_mse_bwd": (c_int, [c_void_p, c_void_p, c_void_p, c_longlong, c_void_p, c_void_p, c_void_p]),
        "dtp_mse_pair_fwd": (c_int, [c_void_p, c_void_p, c_void_p, c_longlong, c_void_p, c_void_p, c_void_p, c_void_p,
                                     c_void_p, c_int, c_void_p]),
        "dtp_mse_pair_bwd": (c_int, [c_void_p] * 6 + [c_longlong] + [c_void_p] * 4),
        "dtp_gather_rows2": (c_int, [c_void_p, c_int, c_void_p, c_int, c_void_p, c_int, c_longlong, c_void_p, c_void_p,
                                     c_void_p]),
        "dtp_gather_rows2_ring": (c_int, [c_void_p, c_int, c_void_p, c_int, c_void_p, c_int, c_int, c_int, c_longlong,
                                          c_void_p, c_void_p, c_void_p]),
        "dtp_gather_ring_max_elems": (c_longlong, []),
        "dtp_gather_rows2_sampler": (c_int, [c_void_p, c_int, c_void_p, c_int, P(SamplerCfg), c_void_p, c_int,
                                             c_longlong, c_void_p, c_void_p, c_void_p]),
        "dtp_format_loss_rows": (c_longlong, [c_void_p, c_int, c_longlong, c_longlong, c_longlong, c_longlong,
                                              c_longlong, c_int, c_void_p, c_longlong]),
        "dtp_format_loss_rows_bound": (c_longlong, [c_int, c_longlong]),
        "dtp_format_loss_rows_jsonl": (c_longlong, [c_void_p, c_int, c_longlong, c_longlong, c_longlong, c_longlong,
                                                    c_longlong, ctypes.c_char_p, c_void_p, c_longlong]),
        "dtp_format_loss_rows_jsonl_bound": (c_longlong, [c_int, c_longlong, c_longlong]),
        "dtp_randperm_fill": (c_int, [ctypes.c_ulonglong, c_int, c_longlong, c_int, c_void_p, c_int]),
        "dtp_split_launch": (c_int, [P(SplitLaunch), c_void_p]),
        "dtp_split_shape_id": (c_int, [c_int] * 6),
        "dtp_split_stage_supported": (c_int, [c_int] * 6),
        "dtp_split_link_bytes": (c_longlong, [c_int, c_int]),
        "dtp_split_lanes_launch": (c_int, [P(SplitLaunch), c_void_p]),
        "dtp_split_lanes_supported": (c_int, [c_int] * 6),
        "dtp_split_lanes_grp_bytes": (c_longlong, [c_int, c_int]),
        "dtp_sampler_indices": (c_int, [P(SamplerCfg), c_longlong, c_int, c_void_p, c_void_p]),
        "dtp_get_device": (c_int, [P(c_int)]),
        "dtp_device_count": (c_int, [P(c_int)]),
        "dtp_malloc_uncached": (c_int, [c_size_t, P(c_void_p)]),
        "dtp_malloc": (c_int, [c_size_t, P(c_void_p)]),
        "dtp_free": (c_int, [c_void_p]),
        "dtp_ipc_handle_size": (c_int, []),
        "dtp_ipc_get_handle": (c_int, [c_void_p, c_void_p]),
        "dtp_ipc_open_handle": (c_int, [c_void_p, P(c_void_p)]),
        "dtp_ipc_close_handle": (c_int, [c_void_p]),
        "dtp_can_access_peer": (c_int, [c_int, c_int, P(c_int)]),
        "dtp_enable_peer_access": (c_int, [c_int]),
        "dtp_memcpy_peer_async": (c_int, [c_void_p, c_int, c_void_p, c_int, c_size_t, c_void_p]),
        "dtp_memcpy_h2d": (c_int, [c_void_p, c_void_p, c_size_t]),
        "dtp_memcpy_d2h": (c_int, [c_void_p, c_void_p, c_size_t]),
        "dtp_stream_sync": (c_int, [c_void_p]),
        "dtp_stream_create_cu_mask": (c_int, [ctypes.POINTER(ctypes.c_uint), c_int, ctypes.POINTER(c_void_p)]),
        "dtp_stream_create_priority": (c_int, [c_int, P(c_void_p)]),
        "dtp_stream_priority_range": (c_int, [P(c_int), P(c_int)]),
        "dtp_stream_destroy": (c_int, [c_void_p]),
        "dtp_device_sync_check": (c_int, []),
        "dtp_graph_capture_train": (c_int, [P(TrainArgs), c_int, c_int, c_int, c_int, c_int, c_int, c_void_p,
                                            P(c_void_p)]),
        "dtp_graph_launch": (c_int, [c_void_p, c_void_p]),
        "dtp_graph_capture_engine": (c_int, [c_void_p, c_int, c_void_p, P(c_void_p)]),
        "dtp_graph_destroy": (c_int, [c_void_p]),
        "dtp_struct_sizes": (c_int, [P(c_int)]),
        "dtp_gemm": (c_int, [P(GemmArgs), c_void_p]),
        "dtp_gemm_workspace": (c_longlong, [P(GemmArgs)]),
        "dtp_xgmi_allreduce": (c_int, [c_void_p, c_int, c_int, c_void_p, c_int, c_int, c_void_p, c_float,
                                       c_void_p, c_int, c_void_p]),
        "dtp_xgmi_allreduce_epoch_slots": (c_int, [c_int]),
        "dtp_colsum": (c_int, [c_void_p, c_longlong, c_int, c_int, c_int, c_void_p, c_int, c_void_p]),
    }
    for name, (res, args) in sig.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args


def load(build_if_missing: bool = False):
    """Load libdtp.so (optionally building it first). Raises NativeUnavailable."""
    global _lib
    if _lib is not None:
        return _lib
    with _lock:
        if _lib is not None:
            return _lib
        if not LIB_PATH.exists() and build_if_missing:
            from . import build as _build

            _build.build()
        if not LIB_PATH.exists():
            raise NativeUnavailable(
                f"{LIB_PATH} is missing: build it with `python -m distributed_training_pytorch_amd.build` "
                "(hipcc --offload-arch=gfx950)")
        try:
            lib = ctypes.CDLL(str(LIB_PATH), mode=ctypes.RTLD_GLOBAL)
        except OSError as e:  # pragma: no cover
            raise NativeUnavailable(f"cannot load {LIB_PATH}: {e}") from e
        _declare(lib)
        sizes = (c_int * 8)()
        lib.dtp_struct_sizes(sizes)
        mine = [ctypes.sizeof(t) for t in (SamplerCfg, Hyper, TrainArgs, StageArgs, OptArgs, GemmArgs, SplitStageArgs,
                                            SplitLaunch)]
        if list(sizes[:8]) != mine:
            raise NativeUnavailable(f"ABI mismatch between libdtp.so {list(sizes[:8])} and _native.py {mine}: rebuild")
        check_stamp(lib)
        _lib = lib
        return lib


def check_stamp(lib) -> None:
    """The library must have been built from the csrc sources next to it: its baked-in
    ``dtp_source_hash()`` is compared with ``build.source_hash()`` of the tree (skipped
    for A/B variant builds loaded through DTP_LIB, and with DTP_SKIP_STAMP=1)."""
    if os.environ.get("DTP_LIB") or os.environ.get("DTP_SKIP_STAMP") == "1":
        return
    from . import build as _build

    if not _build.CSRC.exists():
        return
    have = (lib.dtp_source_hash() or b"").decode()
    want = _build.source_hash()
    if have != want:
        raise NativeUnavailable(f"{LIB_PATH} is stale: built from sources {have}, tree has {want}; rebuild with "
                                "`python -m distributed_training_pytorch_amd.build`")


def source_hash() -> str:
    """Build stamp of the loaded library (``dtp_source_hash``)."""
    return (load().dtp_source_hash() or b"").decode()


def available() -> bool:
    try:
        load()
        return True
    except NativeUnavailable:
        return False


def require(device: torch.device | None = None):
    """Return the library for a GPU op; raise loudly if it cannot be loaded."""
    try:
        return load()
    except NativeUnavailable as e:
        raise NativeUnavailable(f"native HIP kernels are required on {device or 'GPU'}: {e}") from e


def debug_enabled() -> bool:
    """DTP_DEBUG=1: synchronise + error-check after every native call, poison fresh outputs."""
    return os.environ.get("DTP_DEBUG", "0") == "1"


def check(rc: int, what: str):
    if rc != 0:
        lib = load()
        msg = (lib.dtp_last_error() or b"").decode() or (lib.dtp_runtime_last_error() or b"").decode()
        raise RuntimeError(f"{what} failed (rc={rc}): {msg}")
    if debug_enabled():
        lib = load()
        if lib.dtp_device_sync_check() != 0:
            msg = (lib.dtp_runtime_last_error() or b"").decode()
            raise RuntimeError(f"{what}: device fault surfaced by DTP_DEBUG sync: {msg}")


def stream_ptr(stream: torch.cuda.Stream | None = None) -> int:
    """Raw hipStream_t of ``stream`` or of the current device's current stream (the
    capture stream inside ``torch.cuda.graph``).  The default path reads it straight
    from c10: ``torch.cuda.current_stream()`` with no device resolves the device through
    ``torch.cuda.is_available()``, a ``hipGetDeviceCount`` per call (~30 us on the
    MI355X box), which was the largest host cost of every native op launch."""
    if stream is not None:
        return int(stream.cuda_stream)
    return torch._C._cuda_getCurrentRawStream(torch._C._cuda_getDevice())


def raw_stream(device_index: int) -> int:
    """The current stream of a device as a raw hipStream_t (no Stream object built)."""
    return torch._C._cuda_getCurrentRawStream(device_index)


def ptr(t: torch.Tensor | None) -> int | None:
    return None if t is None else int(t.data_ptr())


_WAIT_FLAGS = {"auto": 0x0, "spin": 0x1, "yield": 0x2, "blocking": 0x4}  # hipDeviceSchedule*


def set_wait_mode(mode: str | None = None) -> str:
    """How host threads wait for GPU completion (``hipSetDeviceFlags``).

    ``spin`` keeps the waiting thread polling the completion signal instead of
    sleeping on an interrupt: a ``synchronize`` after a short launch returns a few
    microseconds sooner, at the price of one busy CPU core per rank while it
    waits.  Call before the process touches the GPU.  ``mode=None`` reads
    ``DTP_WAIT_MODE`` (default ``auto``: the runtime's own policy)."""
    mode = mode or os.environ.get("DTP_WAIT_MODE", "auto")
    if mode not in _WAIT_FLAGS:
        raise ValueError(f"wait mode {mode!r} not in {sorted(_WAIT_FLAGS)}")
    if mode == "auto":
        return mode
    hip = ctypes.CDLL("libamdhip64.so.7")  # torch's own runtime (same soname, already loaded)
    rc = hip.hipSetDeviceFlags(ctypes.c_uint(_WAIT_FLAGS[mode]))
    if rc != 0:
        raise RuntimeError(f"hipSetDeviceFlags({mode}) failed with hipError {rc}")
    return mode


def native_enabled() -> bool:
    """DTP_NATIVE=0 forces the PyTorch reference path (debug only; never on a timed run)."""
    return os.environ.get("DTP_NATIVE", "1") != "0"


# streams this module created (raw handle, device index): destroyed at interpreter exit,
# while the HIP runtime is still loaded -- a stream left to the runtime's own teardown
# (its static destructors, after Python has gone) was the suspect of an exit-time
# SIGSEGV in __cxa_finalize under rocprofv3 (profiles/r4_split_streams/README.md)
_owned_streams: list = []
# CU count of every stream made by cu_masked_stream (raw handle -> CUs): a kernel whose
# workgroups must all be resident at once (the split-batch step) checks it
masked_stream_cus: dict[int, int] = {}
_atexit_registered = False


def _own_stream(handle: int, device: torch.device) -> None:
    global _atexit_registered
    _owned_streams.append((handle, device.index if device.index is not None else torch.cuda.current_device()))
    if not _atexit_registered:
        import atexit

        atexit.register(destroy_owned_streams)
        _atexit_registered = True


def destroy_owned_streams() -> None:
    """Synchronise and destroy every stream made by :func:`priority_stream` /
    :func:`cu_masked_stream` (idempotent; registered with atexit)."""
    if not _owned_streams or _lib is None:
        return
    while _owned_streams:
        h, dev = _owned_streams.pop()
        masked_stream_cus.pop(h, None)
        try:
            with torch.cuda.device(dev):
                _lib.dtp_stream_destroy(ctypes.c_void_p(h))
        except Exception:  # noqa: BLE001 - teardown is best effort
            pass


def priority_stream(device, priority: int) -> "torch.cuda.ExternalStream":
    """A torch stream at a HIP stream priority (``hipStreamCreateWithPriority``, lower =
    higher priority); destroyed at interpreter exit (:func:`destroy_owned_streams`)."""
    lib = require(torch.device(device))
    out = ctypes.c_void_p()
    with torch.cuda.device(torch.device(device)):
        check(lib.dtp_stream_create_priority(int(priority), ctypes.byref(out)), "dtp_stream_create_priority")
    _own_stream(out.value, torch.device(device))
    return torch.cuda.ExternalStream(out.value, device=torch.device(device))


def stream_priority_levels(device) -> list[int]:
    """The device's stream priority levels, highest priority first."""
    lib = require(torch.device(device))
    least, greatest = ctypes.c_int(), ctypes.c_int()
    with torch.cuda.device(torch.device(device)):
        check(lib.dtp_stream_priority_range(ctypes.byref(least), ctypes.byref(greatest)), "dtp_stream_priority_range")
    return list(range(greatest.value, least.value + 1))


def cu_masked_stream(device, cus) -> "torch.cuda.ExternalStream":
    """A torch stream whose kernels run only on the listed logical CUs
    (``hipExtStreamCreateWithCUMask``); destroyed at interpreter exit."""
    lib = require(torch.device(device))
    cus = sorted(set(int(c) for c in cus))
    if not cus or cus[0] < 0:
        raise ValueError(f"cu_masked_stream: bad CU list {cus}")
    words = cus[-1] // 32 + 1
    mask = (ctypes.c_uint * words)()
    for c in cus:
        mask[c // 32] |= 1 << (c % 32)
    out = ctypes.c_void_p()
    check(lib.dtp_stream_create_cu_mask(mask, words, ctypes.byref(out)), "dtp_stream_create_cu_mask")
    _own_stream(out.value, torch.device(device))
    masked_stream_cus[out.value] = len(cus)
    return torch.cuda.ExternalStream(out.value, device=torch.device(device))
