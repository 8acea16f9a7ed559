"""ctypes binding of the C-ABI in include/pgmhip.h (libpgmhip.so, gfx950).

This is the seam where pgmpy's numpy/torch dispatch (pgmpy/utils/compat_fns.py:
einsum L63-67, max L53-60, argmax L70-74) is replaced by hand-written HIP
kernels.  There is no CPU fallback: every compute entry point raises
``NativeUnavailable`` when the library or a GPU is missing, so a silent numpy
path can never stand in for the device path.

Device buffers are torch tensors (PyTorch is plumbing here: allocator, streams,
torch.distributed); only raw pointers and the HIP stream handle cross the ABI.
"""
import ctypes
import os
import threading

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("PGM_LIB_PATH") or os.path.join(HERE, "lib", "libpgmhip.so")  # override: tools only

PGM_OK = 0
PGM_EINVAL = -1
PGM_EINDEX = -2
PGM_ENOMEM = -3
PGM_EDEVICE = -4
PGM_MAX_DIMS = 32
PGM_EV_MISSING = 255

COMBINE_MUL, COMBINE_ADD, COMBINE_DIV, COMBINE_COPY, COMBINE_DIV_RAW = 0, 1, 2, 3, 4
RED_NONE, RED_SUM, RED_MAX = 0, 1, 2

ROWS_MAX_LOOP = 12
ROWS_MAX_FAC = 16
ROWS_MAX_EV = 48
ROWS_MAX_COMP = 12
ROWS_MAX_MARG = 192
ROWS_MARGINALS, ROWS_JOINT, ROWS_MAP, ROWS_MAPGAP, ROWS_VALUES_GLOBAL = 1, 2, 4, 8, 16
BATCH_GRID, BATCH_ONE_WORKGROUP = 0, 1  # pgm_batch_set_mode
ROWS_ONE_GROUP, ROWS_GENERIC, ROWS_NO_JIT, ROWS_FLOOR = 32, 64, 128, 256


class NativeUnavailable(RuntimeError):
    """The gfx950 HIP library (or a GPU) is not available: there is no CPU fallback."""


_I64 = ctypes.c_int64 * PGM_MAX_DIMS


class ContractDesc(ctypes.Structure):
    _fields_ = [
        ("combine", ctypes.c_int32),
        ("reduce", ctypes.c_int32),
        ("n_keep", ctypes.c_int32),
        ("n_red", ctypes.c_int32),
        ("keep_card", _I64),
        ("keep_sa", _I64),
        ("keep_sb", _I64),
        ("keep_sc", _I64),
        ("red_card", _I64),
        ("red_sa", _I64),
        ("red_sb", _I64),
    ]


PRODN_MAX_OPS = 8
PM_MAX_OPS = 8  # operands of a fused product + marginal step (pgm_internal.h MOPS)


PRODN_MUL, PRODN_RATIO, PRODN_DEN, PRODN_MDIV = 0, 1, 2, 3


class ProductNDesc(ctypes.Structure):
    _fields_ = [
        ("n_ops", ctypes.c_int32),
        ("n_keep", ctypes.c_int32),
        ("op_kind", ctypes.c_int32 * PRODN_MAX_OPS),
        ("keep_card", _I64),
        ("keep_sc", _I64),
        ("keep_s", _I64 * PRODN_MAX_OPS),
    ]


class ContractNDesc(ctypes.Structure):
    """pgm_contractn_desc (r06): C[keep] = reduce over red of prod_t X_t."""
    _fields_ = [
        ("n_ops", ctypes.c_int32),
        ("reduce", ctypes.c_int32),
        ("n_keep", ctypes.c_int32),
        ("n_red", ctypes.c_int32),
        ("keep_card", _I64),
        ("keep_sc", _I64),
        ("keep_s", _I64 * PRODN_MAX_OPS),
        ("red_card", _I64),
        ("red_s", _I64 * PRODN_MAX_OPS),
    ]


class GemmDesc(ctypes.Structure):
    _fields_ = [("batch", ctypes.c_int64), ("m", ctypes.c_int64), ("n", ctypes.c_int64), ("k", ctypes.c_int64),
                ("offsets", ctypes.c_void_p), ("stride", ctypes.c_int64 * 9), ("lane_order", ctypes.c_int32),
                ("_pad", ctypes.c_int32)]


class GatherDesc(ctypes.Structure):
    _fields_ = [
        ("n_keep", ctypes.c_int32),
        ("n_ev", ctypes.c_int32),
        ("batch_dim", ctypes.c_int32),
        ("_pad", ctypes.c_int32),
        ("ld", ctypes.c_int64),
        ("row0", ctypes.c_int64),
        ("keep_card", _I64),
        ("keep_sa", _I64),
        ("keep_sc", _I64),
        ("ev_col", _I64),
        ("ev_stride", _I64),
        ("ev_card", _I64),
    ]


class RowsPlan(ctypes.Structure):
    _fields_ = [
        ("n_loop", ctypes.c_int32),
        ("n_query", ctypes.c_int32),
        ("n_fac", ctypes.c_int32),
        ("n_ev", ctypes.c_int32),
        ("n_values", ctypes.c_int32),
        ("n_comp", ctypes.c_int32),
        ("n_marg", ctypes.c_int32),
        ("n_joint", ctypes.c_int32),
        ("loop_card", ctypes.c_int32 * ROWS_MAX_LOOP),
        ("loop_marg_off", ctypes.c_int32 * ROWS_MAX_LOOP),
        ("loop_map_stride", ctypes.c_int32 * ROWS_MAX_LOOP),
        ("comp_loop_begin", ctypes.c_int32 * ROWS_MAX_COMP),
        ("comp_n_query", ctypes.c_int32 * ROWS_MAX_COMP),
        ("comp_loop_end", ctypes.c_int32 * ROWS_MAX_COMP),
        ("comp_fac_begin", ctypes.c_int32 * ROWS_MAX_COMP),
        ("comp_fac_end", ctypes.c_int32 * ROWS_MAX_COMP),
        ("fac_base", ctypes.c_int32 * ROWS_MAX_FAC),
        ("fac_stride", (ctypes.c_int32 * ROWS_MAX_LOOP) * ROWS_MAX_FAC),
        ("fac_ev_begin", ctypes.c_int32 * ROWS_MAX_FAC),
        ("fac_ev_end", ctypes.c_int32 * ROWS_MAX_FAC),
        ("ev_col", ctypes.c_int32 * ROWS_MAX_EV),
        ("ev_stride", ctypes.c_int32 * ROWS_MAX_EV),
        ("ev_card", ctypes.c_int32 * ROWS_MAX_EV),
    ]


_P = ctypes.c_void_p
_SIGS = {
    "pgm_version": ([], ctypes.c_int),
    "pgm_last_error": ([ctypes.c_char_p, ctypes.c_size_t], ctypes.c_int),
    "pgm_device_count": ([ctypes.POINTER(ctypes.c_int)], ctypes.c_int),
    "pgm_set_device": ([ctypes.c_int], ctypes.c_int),
    "pgm_alloc": ([ctypes.POINTER(_P), ctypes.c_size_t], ctypes.c_int),
    "pgm_free": ([_P], ctypes.c_int),
    "pgm_memcpy_h2d": ([_P, _P, ctypes.c_size_t, _P], ctypes.c_int),
    "pgm_memcpy_d2h": ([_P, _P, ctypes.c_size_t, _P], ctypes.c_int),
    "pgm_memcpy_d2h_async": ([_P, _P, ctypes.c_size_t, _P], ctypes.c_int),
    "pgm_memcpy_d2d": ([_P, _P, ctypes.c_size_t, _P], ctypes.c_int),
    "pgm_memset": ([_P, ctypes.c_int, ctypes.c_size_t, _P], ctypes.c_int),
    "pgm_host_alloc": ([ctypes.POINTER(_P), ctypes.c_size_t], ctypes.c_int),
    "pgm_host_free": ([_P], ctypes.c_int),
    "pgm_stream_sync_spin": ([_P], ctypes.c_int),
    "pgm_stream_sync": ([_P], ctypes.c_int),
    "pgm_event_create": ([ctypes.POINTER(_P)], ctypes.c_int),
    "pgm_event_destroy": ([_P], ctypes.c_int),
    "pgm_event_record": ([_P, _P], ctypes.c_int),
    "pgm_event_elapsed_ms": ([_P, _P, ctypes.POINTER(ctypes.c_float)], ctypes.c_int),
    "pgm_contract_workspace": ([ctypes.POINTER(ContractDesc), ctypes.POINTER(ctypes.c_size_t)], ctypes.c_int),
    "pgm_contract": ([ctypes.POINTER(ContractDesc), _P, _P, _P, _P, ctypes.c_size_t, _P], ctypes.c_int),
    "pgm_product_n": ([ctypes.POINTER(ProductNDesc), ctypes.POINTER(_P), _P, _P], ctypes.c_int),
    "pgm_product_n_marginal_ok": ([ctypes.POINTER(ProductNDesc), ctypes.POINTER(_P), _P,
                                   ctypes.POINTER(ctypes.c_int64), _P], ctypes.c_int),
    "pgm_product_n_marginal": ([ctypes.POINTER(ProductNDesc), ctypes.POINTER(_P), _P,
                                ctypes.POINTER(ctypes.c_int64), ctypes.c_int32, _P, _P], ctypes.c_int),
    "pgm_product_n_marginal_bind": ([ctypes.POINTER(ProductNDesc), ctypes.POINTER(_P), _P,
                                     ctypes.POINTER(ctypes.c_int64), ctypes.c_int32, _P, ctypes.POINTER(_P)],
                                    ctypes.c_int),
    "pgm_product_n_marginal_source": ([ctypes.POINTER(ProductNDesc), ctypes.POINTER(_P), _P,
                                       ctypes.POINTER(ctypes.c_int64), ctypes.c_int32, _P, ctypes.c_char_p,
                                       ctypes.c_size_t], ctypes.c_int),
    "pgm_product_n_marginals_bind": ([ctypes.POINTER(ProductNDesc), ctypes.POINTER(_P),
                                      ctypes.POINTER(ctypes.c_int64), _P, ctypes.POINTER(ctypes.c_int64), _P,
                                      ctypes.c_int32, ctypes.POINTER(_P)], ctypes.c_int),
    "pgm_product_n_bind": ([ctypes.POINTER(ProductNDesc), ctypes.POINTER(_P), _P, ctypes.POINTER(_P)], ctypes.c_int),
    "pgm_pm_bound_run": ([_P, _P], ctypes.c_int),
    "pgm_pm_merge": ([ctypes.POINTER(_P), ctypes.c_int32, ctypes.POINTER(_P)], ctypes.c_int),
    "pgm_pm_prepare": ([ctypes.POINTER(_P), ctypes.c_int32], ctypes.c_int),
    "pgm_pm_bound_source": ([_P, ctypes.c_char_p, ctypes.c_size_t], ctypes.c_int),
    "pgm_pm_bound_destroy": ([_P], ctypes.c_int),
    "pgm_gemm": ([ctypes.POINTER(GemmDesc), _P, _P, _P, _P], ctypes.c_int),
    "pgm_batch_create": ([ctypes.POINTER(_P)], ctypes.c_int),
    "pgm_batch_add_contract": ([_P, ctypes.POINTER(ContractDesc), _P, _P, _P], ctypes.c_int),
    "pgm_batch_add_gather": ([_P, ctypes.POINTER(GatherDesc), _P, _P, _P, _P], ctypes.c_int),
    "pgm_batch_add_product_n": ([_P, ctypes.POINTER(ProductNDesc), ctypes.POINTER(_P), _P], ctypes.c_int),
    "pgm_batch_add_contract_n": ([_P, ctypes.POINTER(ContractNDesc), ctypes.POINTER(_P), _P], ctypes.c_int),
    "pgm_batch_add_indicator": ([_P, _P, ctypes.c_int64, ctypes.c_int64, _P, ctypes.c_int64, ctypes.c_int64, _P],
                                ctypes.c_int),
    "pgm_batch_set_mode": ([_P, ctypes.c_int32], ctypes.c_int),
    "pgm_batch_blocks": ([_P, ctypes.POINTER(ctypes.c_int64)], ctypes.c_int),
    "pgm_batch_add_level": ([_P], ctypes.c_int),
    "pgm_batch_finalize": ([_P], ctypes.c_int),
    "pgm_batch_run": ([_P, _P], ctypes.c_int),
    "pgm_batch_destroy": ([_P], ctypes.c_int),
    "pgm_batch_specialise": ([_P, ctypes.POINTER(_P)], ctypes.c_int),
    "pgm_codes_select": ([_P, ctypes.c_int64, ctypes.c_int64, _P, ctypes.c_int32, ctypes.c_int64, _P, _P],
                         ctypes.c_int),
    "pgm_graph_capture_begin": ([_P], ctypes.c_int),
    "pgm_graph_capture_end": ([_P, ctypes.POINTER(_P)], ctypes.c_int),
    "pgm_graph_launch": ([_P, _P], ctypes.c_int),
    "pgm_graph_destroy": ([_P], ctypes.c_int),
    "pgm_gather": ([ctypes.POINTER(GatherDesc), _P, _P, _P, _P, _P], ctypes.c_int),
    "pgm_indicator": ([_P, ctypes.c_int64, ctypes.c_int64, _P, ctypes.c_int64, ctypes.c_int64, _P, _P],
                      ctypes.c_int),
    "pgm_argmax": ([_P, ctypes.c_int64, ctypes.c_int64, ctypes.c_int64, ctypes.c_int64, _P, _P, _P], ctypes.c_int),
    "pgm_rows_plan_create": ([ctypes.POINTER(RowsPlan), _P, ctypes.POINTER(_P)], ctypes.c_int),
    "pgm_rows_plan_destroy": ([_P], ctypes.c_int),
    "pgm_rows_plan_run": ([_P, ctypes.c_int32, _P, ctypes.c_int64, ctypes.c_int64, ctypes.c_int64, _P, _P,
                           ctypes.c_int64, _P, _P, _P, _P], ctypes.c_int),
    "pgm_rows_plan_bind": ([_P, ctypes.c_int32, _P, ctypes.c_int64, ctypes.c_int64, ctypes.c_int64, _P, _P,
                            ctypes.c_int64, _P, _P, _P, _P, ctypes.POINTER(ctypes.c_void_p)], ctypes.c_int),
    "pgm_rows_bound_run": ([_P], ctypes.c_int),
    "pgm_rows_plan_source": ([ctypes.c_void_p, ctypes.c_char_p, ctypes.c_size_t, ctypes.POINTER(ctypes.c_size_t)],
                             ctypes.c_int),
    "pgm_rows_bound_destroy": ([_P], ctypes.c_int),
    "pgm_rows_bound_kernel": ([_P, ctypes.c_char_p, ctypes.c_size_t, ctypes.POINTER(ctypes.c_uint32),
                               ctypes.POINTER(ctypes.c_uint32)], ctypes.c_int),
    "pgm_rows_shard_run": ([ctypes.POINTER(_P), ctypes.c_int32, ctypes.c_int32, _P, ctypes.c_int64, ctypes.c_int64,
                            ctypes.c_int64, _P, ctypes.c_int64, _P, _P], ctypes.c_int),
    "pgm_host_any_negative_i8": ([ctypes.POINTER(_P), ctypes.c_int32, ctypes.c_int64, _P, ctypes.c_int32], ctypes.c_int),
    "pgm_host_scan_begin": ([ctypes.c_int64, ctypes.c_int32, ctypes.c_int32, ctypes.POINTER(_P)], ctypes.c_int),
    "pgm_host_scan_push": ([_P, ctypes.POINTER(_P), ctypes.c_int32], ctypes.c_int),
    "pgm_host_scan_end": ([_P, _P, ctypes.POINTER(ctypes.c_int32)], ctypes.c_int),
    "pgm_host_lut_map_u8": ([ctypes.POINTER(_P), ctypes.POINTER(_P), ctypes.c_int32, ctypes.c_int64, _P, ctypes.c_int64,
                             ctypes.c_int32], ctypes.c_int),
    "pgm_rows_ring_create": ([_P, ctypes.c_int32, ctypes.c_int32, ctypes.POINTER(_P), ctypes.POINTER(ctypes.c_int64),
                              ctypes.POINTER(ctypes.c_int64), ctypes.c_int64, ctypes.POINTER(_P), ctypes.c_int64,
                              ctypes.POINTER(_P), ctypes.POINTER(_P), _P, _P, ctypes.POINTER(ctypes.c_void_p)],
                             ctypes.c_int),
    "pgm_rows_ring_start": ([_P, ctypes.c_uint32, ctypes.c_double], ctypes.c_int),
    "pgm_rows_ring_start_ready": ([_P, ctypes.c_uint32, ctypes.c_double, ctypes.c_double], ctypes.c_int),
    "pgm_rows_ring_post": ([_P, ctypes.c_uint32], ctypes.c_int),
    "pgm_rows_ring_finish": ([_P], ctypes.c_int),
    "pgm_rows_ring_cancel": ([_P], ctypes.c_int),
    "pgm_rows_ring_counter": ([_P, ctypes.POINTER(ctypes.c_void_p), ctypes.POINTER(ctypes.c_uint32)], ctypes.c_int),
    "pgm_rows_ring_kernel": ([_P, ctypes.c_char_p, ctypes.c_size_t, ctypes.POINTER(ctypes.c_uint32),
                              ctypes.POINTER(ctypes.c_uint32)], ctypes.c_int),
    "pgm_rows_ring_destroy": ([_P], ctypes.c_int),
    "pgm_codes_remap": ([_P, ctypes.c_int64, ctypes.c_int32, ctypes.c_int64, _P, ctypes.c_int32, _P, _P,
                         ctypes.c_int64, _P, _P, _P, _P, _P], ctypes.c_int),
    "pgm_sample_joint": ([_P, ctypes.c_int64, ctypes.c_int64, _P, _P, ctypes.c_int64, _P, _P], ctypes.c_int),
    "pgm_dq_create": ([ctypes.c_int, ctypes.POINTER(ctypes.c_void_p)], ctypes.c_int),
    "pgm_dq_destroy": ([_P], ctypes.c_int),
    "pgm_dq_bind_rows": ([_P, _P, ctypes.POINTER(ctypes.c_void_p)], ctypes.c_int),
    "pgm_dq_launch": ([_P], ctypes.c_int),
    "pgm_dq_launch_group": ([ctypes.POINTER(ctypes.c_void_p), ctypes.c_int32], ctypes.c_int),
    "pgm_dq_sync": ([_P], ctypes.c_int),
    "pgm_dq_wait": ([_P], ctypes.c_int),
    "pgm_dq_release": ([_P], ctypes.c_int),
    "pgm_dq_launch_release": ([_P], ctypes.c_int),
    "pgm_dq_timer_start": ([_P], ctypes.c_int),
    "pgm_dq_timer_stop_ms": ([_P, ctypes.POINTER(ctypes.c_float)], ctypes.c_int),
    "pgm_dq_timer_stop_ticks": ([_P, ctypes.POINTER(ctypes.c_uint64), ctypes.POINTER(ctypes.c_uint64),
                                 ctypes.POINTER(ctypes.c_uint64)], ctypes.c_int),
    "pgm_dq_timer_dispatch_stats": ([_P, ctypes.POINTER(ctypes.c_uint64), ctypes.POINTER(ctypes.c_uint64)],
                                    ctypes.c_int),
    "pgm_dq_bound_destroy": ([_P], ctypes.c_int),
    "pgm_dq_bind_pm": ([_P, _P, ctypes.POINTER(ctypes.c_void_p)], ctypes.c_int),
    "pgm_dq_run_chain": ([ctypes.POINTER(ctypes.c_void_p), ctypes.POINTER(ctypes.c_uint8), ctypes.c_int32],
                         ctypes.c_int),
    "pgm_dq_profiling": ([_P, ctypes.c_int32], ctypes.c_int),
    "pgm_dq_timer_dispatch_times": ([_P, ctypes.POINTER(ctypes.c_uint64), ctypes.POINTER(ctypes.c_uint64),
                                     ctypes.c_int32, ctypes.POINTER(ctypes.c_int32)], ctypes.c_int),
}

EXPORTED = tuple(_SIGS)

_lock = threading.Lock()
_lib = None
_device_ok = None


def load_library():
    """Load libpgmhip.so (no GPU needed). Raises NativeUnavailable if it was not built."""
    global _lib
    with _lock:
        if _lib is not None:
            return _lib
        if not os.path.exists(LIB_PATH):
            raise NativeUnavailable(
                f"{LIB_PATH} is missing: build it with `python -m pgmpy_amd.build` (hipcc --offload-arch=gfx950)")
        lib = ctypes.CDLL(LIB_PATH)
        for name, (argtypes, restype) in _SIGS.items():
            fn = getattr(lib, name)
            fn.argtypes = argtypes
            fn.restype = restype
        _lib = lib
        return lib


def last_error():
    lib = load_library()
    buf = ctypes.create_string_buffer(1024)
    lib.pgm_last_error(buf, len(buf))
    return buf.value.decode(errors="replace")


def check(rc, what=""):
    if rc == PGM_OK:
        return
    msg = f"{what}: {last_error()}" if what else last_error()
    if rc == PGM_EINVAL:
        raise ValueError(msg)
    if rc == PGM_EINDEX:
        raise IndexError(msg)
    if rc == PGM_ENOMEM:
        raise MemoryError(msg)
    raise RuntimeError(msg)


def lib():
    """The library, for compute: additionally requires a visible GPU (no CPU fallback)."""
    global _device_ok
    L = load_library()
    if _device_ok is None:
        import torch

        _device_ok = bool(torch.cuda.is_available())
    if not _device_ok:
        raise NativeUnavailable("no HIP device visible: the gfx950 kernels need an MI355X (no CPU fallback)")
    return L


def stream_handle(stream=None):
    import torch

    s = stream if stream is not None else torch.cuda.current_stream()
    return ctypes.c_void_p(s.cuda_stream)


class _HostBytes:
    """Owner of one pinned host allocation (pgm_host_alloc), exported through __array_interface__:
    numpy arrays made from it (and their views) reference it, so the memory is freed by reference
    counting as soon as the last of them is gone (no cycle back to the HostBuffer)."""

    def __init__(self, ptr, nbytes):
        self._p = ctypes.c_void_p(ptr)
        self.__array_interface__ = {"data": (ptr, False), "shape": (nbytes,), "typestr": "|u1", "version": 3}

    def __del__(self):
        p = getattr(self, "_p", None)
        if p is not None and p.value:
            try:
                load_library().pgm_host_free(p)
            except Exception:
                pass
            self._p = None


class HostBuffer:
    """Pinned, mapped, coherent host memory that kernels read and write directly (pgm_host_alloc):
    `array` (numpy) and `tensor` (a CPU torch view of the same bytes, for descriptor building) share
    it; the memory belongs to the _HostBytes object the arrays are based on and is freed once the
    HostBuffer and every array / tensor viewing it are gone."""

    def __init__(self, shape, dtype):
        import torch

        L = lib()
        dtype = np.dtype(dtype)
        n = int(np.prod(shape)) if len(shape) else 1
        p = ctypes.c_void_p()
        nbytes = max(1, n * dtype.itemsize)
        check(L.pgm_host_alloc(ctypes.byref(p), nbytes), "host_alloc")
        raw = np.asarray(_HostBytes(p.value, nbytes))
        self.array = raw[:n * dtype.itemsize].view(dtype).reshape(shape)
        self.tensor = torch.from_numpy(self.array)


def ptr(t):
    """Raw device pointer of a torch tensor (or None)."""
    if t is None:
        return None
    return ctypes.c_void_p(t.data_ptr())


def i64arr(vals):
    a = _I64()
    for i, v in enumerate(vals):
        a[i] = int(v)
    return a
