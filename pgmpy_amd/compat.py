"""The "hip" compute backend at the reference's own operator seam.

pgmpy routes every factor operation through two places:

* ``pgmpy.config`` (``pgmpy/global_vars.py:82-122``): ``set_backend("numpy" | "torch")`` decides
  what ``DiscreteFactor.values`` is (``DiscreteFactor.py:94-102``, ``CPD.py:154-161``);
* ``pgmpy/utils/compat_fns.py``: ``einsum`` (L63-67), ``max`` (L53-60), ``argmax`` (L70-74),
  ``size``, ``copy``, ``tobytes``, ``to_numpy``, ``ravel_f``, ``ones``, ``get_compute_backend`` ...,
  plus plain array arithmetic on ``values`` inside DiscreteFactor: ``values / values.sum()``
  (normalize, L530), ``values[tuple(slice_)]`` (reduce, L614), ``values[..., np.newaxis]`` +
  ``swapaxes`` + ``+`` (sum, L690-712), ``values *= k`` (scalar product, L765-766), ``/`` then
  ``values[isnan(values)] = 0`` (divide, L835-863).

This module is what a ``"hip"`` backend plugs into that seam: :class:`Config` accepts
``set_backend("hip")``, :class:`HipArray` is the ``values`` type (an fp64 device array whose views
— indexing, ``np.newaxis``, ``swapaxes``, ``reshape`` — are strided metadata and whose arithmetic
and reductions are single ``pgm_contract`` calls of the C-ABI), and the functions below keep the
exact signatures of ``compat_fns``.  INTEGRATION.md shows the few lines a maintainer adds to
pgmpy to select it.  There is no CPU path: every computing call goes to libpgmhip and raises
``NativeUnavailable`` without it.
"""
import builtins
import numbers

import numpy as np

from . import _native as N
from . import engine as E

BACKENDS = ("numpy", "torch", "hip")


class Config:
    """``pgmpy.global_vars.Config`` with the "hip" backend (global_vars.py:82-122): the backend
    name, the device (the HIP device the values live on) and the dtype (fp64 only on "hip",
    global_vars.py:38)."""

    def __init__(self):
        self.BACKEND = "numpy"
        self.DEVICE = None
        self.DTYPE = "float64"
        self.SHOW_PROGRESS = True

    def set_backend(self, backend, device=None, dtype=None):
        if backend not in BACKENDS:
            raise ValueError(f"backend can either be `numpy`, `torch` or `hip`. Got: {backend}")
        self.BACKEND = backend
        if backend == "numpy":
            self.DEVICE = None
        elif backend == "hip":
            N.lib()  # fails loudly without the library or a device
            import torch

            if device is not None and not str(device).startswith("cuda"):
                raise ValueError(f"the hip backend runs on a HIP device ('cuda' / 'cuda:x'). Got: {device}")
            self.DEVICE = torch.device(device) if device is not None else torch.device("cuda", torch.cuda.current_device())
        else:
            import torch

            self.DEVICE = torch.device(device) if device is not None else (
                torch.device("cuda:0") if torch.cuda.is_available() else torch.device("cpu"))
        self.set_dtype(dtype)

    def get_backend(self):
        return self.BACKEND

    def set_device(self, device=None):
        if self.BACKEND == "hip":
            self.set_backend("hip", device=device, dtype=self.DTYPE)
        else:
            self.DEVICE = device

    def get_device(self):
        return self.DEVICE

    def set_dtype(self, dtype=None):
        if dtype is None:
            dtype = "float64"
        name = str(getattr(dtype, "name", dtype)).replace("torch.", "")
        if self.BACKEND == "hip" and name != "float64":
            raise ValueError(f"the hip backend computes in float64 (pgmpy's default dtype). Got: {dtype}")
        self.DTYPE = name

    def get_dtype(self):
        return self.DTYPE

    def set_show_progress(self, show_progress):
        self.SHOW_PROGRESS = bool(show_progress)

    def get_show_progress(self):
        return self.SHOW_PROGRESS


config = Config()


def _labels(n):
    return list(range(n))


class _NanMask:
    """``isnan(values)`` of a HipArray; only ``values[mask] = 0`` is supported (divide, L859-863)."""

    def __init__(self, arr):
        self.arr = arr


class HipArray:
    """fp64 device array: the ``values`` of a DiscreteFactor under the "hip" backend.

    Wraps a strided torch tensor (device memory from the caching allocator; torch is plumbing).
    Views change strides only; every arithmetic operation or reduction is one pgm_contract call
    with numpy broadcasting expressed as stride-0 operands."""

    __array_priority__ = 1000  # numpy defers binary operators to us

    def __init__(self, t):
        self.t = t

    # ------------------------------------------------------------------ construction / host
    @classmethod
    def from_host(cls, values, shape=None):
        a = np.asarray(values, dtype=np.float64)
        if shape is not None:
            a = a.reshape(shape)
        return cls(E.to_device(a))

    def __array__(self, dtype=None, copy=None):
        a = E.to_host(self.t)
        return a if dtype is None else a.astype(dtype)

    def __repr__(self):
        return f"HipArray({np.asarray(self)!r})"

    def __float__(self):
        if self.t.numel() != 1:
            raise TypeError("only single-element arrays convert to float")
        return float(np.asarray(self).reshape(-1)[0])

    # ------------------------------------------------------------------ metadata
    @property
    def shape(self):
        return tuple(int(s) for s in self.t.shape)

    @property
    def ndim(self):
        return self.t.dim()

    @property
    def size(self):
        return int(self.t.numel())

    def nelement(self):
        return int(self.t.numel())

    def dim(self):
        return self.t.dim()

    @property
    def dtype(self):
        return np.dtype(np.float64)

    # ------------------------------------------------------------------ views (no data movement)
    def reshape(self, *shape):
        shape = tuple(shape[0]) if len(shape) == 1 and not isinstance(shape[0], numbers.Integral) else shape
        t = self.t if self.t.is_contiguous() else E.copy(self.t)
        return HipArray(t.reshape(tuple(int(s) for s in shape)))

    def swapaxes(self, a, b):
        return HipArray(self.t.transpose(int(a), int(b)))

    def transpose(self, axes=None):
        axes = list(reversed(range(self.ndim))) if axes is None else [int(x) for x in axes]
        return HipArray(self.t.permute(*axes))

    def __getitem__(self, key):
        """Basic indexing: ints, slices, ``np.newaxis`` / None, Ellipsis (reduce, L614; the
        broadcast axes of sum / divide, L697-699, L842-844) — a strided view."""
        if isinstance(key, _NanMask):
            raise TypeError("boolean-mask reads are not supported on the hip backend")
        if not isinstance(key, tuple):
            key = (key,)
        norm = []
        for k in key:
            if isinstance(k, (numbers.Integral, np.integer)) and not isinstance(k, bool):
                norm.append(int(k))
            elif k is None or isinstance(k, slice) or k is Ellipsis:
                norm.append(k)
            else:
                raise IndexError(f"only integers, slices, None and Ellipsis index a HipArray, got {type(k)}")
        dims = [d for d, k in enumerate(norm) if isinstance(k, int)]
        shape = self.shape
        for d in dims:  # numpy's IndexError for an out-of-range state (test_Factor.py:555-565)
            ax = builtins.sum(1 for k in norm[:d] if k is not None and k is not Ellipsis)
            if ax < len(shape) and not -shape[ax] <= norm[d] < shape[ax]:
                raise IndexError(f"index {norm[d]} is out of bounds for axis {ax} with size {shape[ax]}")
        return HipArray(self.t[tuple(norm)])

    def __setitem__(self, key, value):
        if isinstance(key, _NanMask) and key.arr.t.data_ptr() == self.t.data_ptr() and float(value) == 0.0:
            # values[isnan(values)] = 0 (DiscreteFactor.py:863): NaN -> 0 in place, IEEE inf kept
            la = _labels(self.ndim)
            one = _scalar(1.0)
            E.contract(self.t, la, one, [], la, combine="div", out=self.t)
            return
        raise TypeError("only values[isnan(values)] = 0 assigns into a HipArray")

    # ------------------------------------------------------------------ arithmetic
    def _binary(self, other, combine, reverse=False):
        a, b = (other, self) if reverse else (self, other)
        ta, tb = _as_tensor(a), _as_tensor(b)
        out_shape = np.broadcast_shapes(tuple(ta.shape), tuple(tb.shape))
        nd = len(out_shape)
        out_l = _labels(nd)

        def fit(t):  # right-align like numpy; size-1 axes that broadcast drop out (stride 0)
            off = nd - t.dim()
            keep = [d for d in range(t.dim()) if t.shape[d] == out_shape[off + d]]
            for d in reversed(range(t.dim())):
                if d not in keep:
                    t = t.squeeze(d)
            return t, [off + d for d in keep]

        (ta, la), (tb, lb) = fit(ta), fit(tb)
        return HipArray(E.contract(ta, la, tb, lb, out_l, combine=combine))

    def __mul__(self, other):
        return self._binary(other, "mul")

    __rmul__ = __mul__

    def __imul__(self, other):
        # values *= k (DiscreteFactor.py:765-766): in place when the result keeps the shape
        if isinstance(other, numbers.Number) or (isinstance(other, HipArray) and other.size == 1):
            la = _labels(self.ndim)
            E.contract(self.t, la, _as_tensor(other).reshape(()), [], la, combine="mul", out=self.t)
            return self
        return self._binary(other, "mul")

    def __truediv__(self, other):
        return self._binary(other, "div_raw")  # IEEE: 0/0 = NaN, x/0 = inf, as numpy

    def __rtruediv__(self, other):
        return self._binary(other, "div_raw", reverse=True)

    def __add__(self, other):
        return self._binary(other, "add")

    __radd__ = __add__

    def __iadd__(self, other):
        return self._binary(other, "add")

    def __rsub__(self, other):
        """``1 - values`` (the virtual-evidence child CPD, inference/base.py:286): other + (-1) * values."""
        neg = self._binary(-1.0, "mul")
        return neg._binary(other, "add")

    def __neg__(self):
        return self._binary(-1.0, "mul")

    # ------------------------------------------------------------------ reductions
    def sum(self, axis=None):
        return HipArray(_reduce(self, axis, "sum"))

    def max(self, axis=None):
        return HipArray(_reduce(self, axis, "max"))

    def flatten(self):
        """``values.flatten()`` (is_valid_cpd, DiscreteFactor.py:959-964): a contiguous 1-D array."""
        return self.reshape(self.size)

    ravel = flatten


def _as_tensor(x):
    if isinstance(x, HipArray):
        return x.t
    if isinstance(x, numbers.Number):
        return _scalar(x)
    return E.to_device(np.asarray(x, dtype=np.float64))


def _scalar(x):
    return E.scalar(float(x)).reshape(())  # a 0-d device value (broadcasts over every axis)


def _reduce(arr, axis, how):
    la = _labels(arr.ndim)
    if axis is None:
        keep = []
    else:
        ax = {int(a) % arr.ndim for a in (axis if isinstance(axis, (tuple, list)) else (axis,))}
        keep = [l for l in la if l not in ax]
    if len(keep) == arr.ndim:
        return E.copy(arr.t)
    return E.contract(arr.t, la, None, None, keep, reduce=how, combine="copy")


# ---------------------------------------------------------------------- compat_fns signatures
def size(arr):
    """compat_fns.size (L21-25)."""
    return arr.size if isinstance(arr, (np.ndarray, HipArray)) else arr.nelement()


def copy(arr):
    """compat_fns.copy (L28-42): a device copy on the hip backend."""
    if isinstance(arr, HipArray):
        return HipArray(E.copy(arr.t))
    if isinstance(arr, (int, float)):
        return arr
    return HipArray.from_host(arr)


def tobytes(arr):
    """compat_fns.tobytes (L45-49) — hashing a factor downloads its values."""
    return np.asarray(arr).tobytes()


def max(arr, axis=None):
    """compat_fns.max (L53-60): np.max over `axis` (NaN propagates, as np.max) — one pgm_contract
    (COPY, MAX)."""
    if not isinstance(arr, HipArray):
        return np.max(arr, axis=None if axis is None else tuple(axis))
    return HipArray(_reduce(arr, None if axis is None else tuple(axis), "max"))


def einsum(*args):
    """compat_fns.einsum (L63-67) in the sublist form pgmpy calls: ``einsum(A, ia, out)``
    (marginalize, DiscreteFactor.py:408) and ``einsum(A, ia, B, ib, out)`` (product, L771-777)."""
    if len(args) == 3:
        A, ia, out = args
        return HipArray(E.contract(_as_tensor(A), list(ia), None, None, list(out), reduce="sum", combine="copy"))
    if len(args) == 5:
        A, ia, B, ib, out = args
        return HipArray(E.contract(_as_tensor(A), list(ia), _as_tensor(B), list(ib), list(out), reduce="sum",
                                   combine="mul"))
    raise ValueError("the hip backend's einsum takes the sublist forms (A, ia, out) or (A, ia, B, ib, out)")


def argmax(arr):
    """compat_fns.argmax (L70-74): np.argmax's first flat index (NaN first), ExactInference.py:616."""
    if not isinstance(arr, HipArray):
        return np.argmax(arr)
    return int(E.to_host(E.argmax_rows(arr.t, _labels(arr.ndim)).double())[0])


def stack(arr_iter):
    """compat_fns.stack (L77-81)."""
    arrs = [np.asarray(a) for a in arr_iter]
    return HipArray.from_host(np.stack(arrs))


def to_numpy(arr, decimals=None):
    """compat_fns.to_numpy (L84-95)."""
    a = np.array(arr)
    return a if decimals is None else a.round(decimals)


def ravel_f(arr):
    """compat_fns.ravel_f (L98-102)."""
    return np.asarray(arr).ravel("F")


def ones(n):
    """compat_fns.ones (L105-110)."""
    return HipArray.from_host(np.ones(n)) if config.get_backend() == "hip" else np.ones(n, dtype=config.get_dtype())


def transpose(arr, axis):
    """compat_fns.transpose."""
    return arr.transpose(axis) if isinstance(arr, HipArray) else np.transpose(arr, axis)


def isnan(arr):
    return _NanMask(arr) if isinstance(arr, HipArray) else np.isnan(arr)


def _is_torch(x):
    try:
        import torch
    except ImportError:  # pragma: no cover
        return False
    return isinstance(x, torch.Tensor)


def _host(x):
    if isinstance(x, HipArray):
        return np.asarray(x)
    if _is_torch(x):
        return x.detach().cpu().numpy()
    return np.asarray(x)


def unique(arr, axis=0, return_counts=False, return_inverse=False):
    """compat_fns.unique (L123-131).  Its callers (sampling/base.py:148) use the results as host
    bookkeeping, so a HipArray is reduced on the host (numpy's semantics)."""
    if _is_torch(arr):
        import torch

        return torch.unique(arr, return_inverse=return_inverse, return_counts=return_counts, dim=axis)
    return np.unique(_host(arr), axis=axis, return_counts=return_counts, return_inverse=return_inverse)


def flip(arr, axis=0):
    """compat_fns.flip (L134-138): assignment() flips its integer index table (DiscreteFactor.py:312)."""
    if isinstance(arr, np.ndarray):
        return np.flip(arr, axis=axis)
    dims = tuple(axis) if isinstance(axis, (tuple, list)) else (int(axis),)
    if isinstance(arr, HipArray):
        return HipArray(arr.t.flip(dims))
    import torch

    return torch.flip(arr, dims=dims)


def exp(arr):
    """compat_fns.exp (L148-152) — elementwise, off the hot path (MirrorDescentEstimator)."""
    if isinstance(arr, HipArray):
        return HipArray(arr.t.exp())
    if isinstance(arr, np.ndarray):
        return np.exp(arr)
    return arr.exp()


def sum(arr):
    """compat_fns.sum (L155-159): the partition function's total (DiscreteMarkovNetwork.py:844,
    ClusterGraph.py:327) — one pgm_contract reduction to a scalar on the hip backend."""
    if isinstance(arr, HipArray):
        return float(HipArray(_reduce(arr, None, "sum")))
    if isinstance(arr, np.ndarray):
        return arr.sum()
    import torch

    return torch.sum(arr)


def allclose(arr1, arr2, atol):
    """compat_fns.allclose (L162-186) with numpy's tolerance rule (rtol 1e-5 + atol): DiscreteFactor.__eq__
    (L1079) and is_valid_cpd (L959).  A comparison verdict, not a hot-path value: compared on the host."""
    return bool(np.allclose(_host(arr1), _host(arr2), atol=atol))


class _HipCompute:
    """What compat_fns.get_compute_backend() returns on the hip backend: the array-namespace calls
    pgmpy makes through it — ``isnan`` (divide, DiscreteFactor.py:863), ``zeros`` (assignment's
    integer table, L304-306: a torch integer tensor on the HIP device, as the torch backend builds
    it next to the torch index of L293-298), ``allclose`` (is_valid_cpd, L959) and ``vstack`` (the
    virtual-evidence CPD, inference/base.py:286)."""

    isnan = staticmethod(isnan)

    @staticmethod
    def zeros(shape, dtype=int):
        import torch

        tdt = torch.int64 if dtype in (int, np.int64, "int64") else torch.float64
        return torch.zeros(shape, dtype=tdt, device=config.get_device())

    @staticmethod
    def allclose(a, b, atol=1e-08, rtol=1e-05):
        return bool(np.allclose(_host(a), _host(b), atol=atol, rtol=rtol))

    @staticmethod
    def vstack(arrs):
        parts = [_host(a) for a in arrs]
        return HipArray.from_host(np.vstack(parts))


def get_compute_backend():
    """compat_fns.get_compute_backend (L113-120)."""
    if config.get_backend() == "hip":
        return _HipCompute
    if config.get_backend() == "numpy":
        return np
    import torch

    return torch


def values_array(values, cardinality):
    """What DiscreteFactor.__init__ / TabularCPD build for ``values`` on the hip backend
    (DiscreteFactor.py:94-102 for numpy / torch)."""
    return HipArray.from_host(values, tuple(int(c) for c in cardinality))
