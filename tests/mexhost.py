"""Call the vlgba MEX gateways (matlab/*.mexa64) from Python through the
repository's mx runtime (matlab/mx_host.c -> libvlgmx.so): numpy arrays in,
MATLAB-shaped numpy arrays out, exactly as MATLAB would pass them."""
import ctypes
import os

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
MATLAB = os.path.join(ROOT, "matlab")
_mx = None
_gw = {}
GATEWAY_T = ctypes.CFUNCTYPE(None, ctypes.c_int, ctypes.POINTER(ctypes.c_void_p), ctypes.c_int,
                             ctypes.POINTER(ctypes.c_void_p))


def mx():
    global _mx
    if _mx is None:
        L = ctypes.CDLL(os.path.join(MATLAB, "libvlgmx.so"), mode=ctypes.RTLD_GLOBAL)
        L.mxhost_double.restype = ctypes.c_void_p
        L.mxhost_double.argtypes = [ctypes.c_int, ctypes.POINTER(ctypes.c_longlong),
                                    ctypes.c_void_p]
        L.mxhost_struct.restype = ctypes.c_void_p
        L.mxhost_set_field.argtypes = [ctypes.c_void_p, ctypes.c_char_p, ctypes.c_void_p]
        L.mxhost_dims.argtypes = [ctypes.c_void_p, ctypes.POINTER(ctypes.c_longlong)]
        L.mxGetPr.restype = ctypes.c_void_p
        L.mxGetPr.argtypes = [ctypes.c_void_p]
        L.mxGetNumberOfElements.restype = ctypes.c_size_t
        L.mxGetNumberOfElements.argtypes = [ctypes.c_void_p]
        L.mxDestroyArray.argtypes = [ctypes.c_void_p]
        L.mxhost_call.argtypes = [ctypes.c_void_p, ctypes.c_int,
                                  ctypes.POINTER(ctypes.c_void_p), ctypes.c_int,
                                  ctypes.POINTER(ctypes.c_void_p), ctypes.c_char_p, ctypes.c_int]
        _mx = L
    return _mx


def gateway(name):
    """mexFunction of matlab/<name>.mexa64 (loaded after libvlgmx)."""
    if name not in _gw:
        mx()
        L = ctypes.CDLL(os.path.join(MATLAB, name + ".mexa64"))
        _gw[name] = (L, ctypes.cast(L.mexFunction, ctypes.c_void_p))
    return _gw[name][1]


def to_mx(v):
    """numpy array / scalar -> mxArray* (double, column major); dict -> 1x1 struct."""
    L = mx()
    if isinstance(v, dict):
        s = L.mxhost_struct()
        for k, f in v.items():
            L.mxhost_set_field(s, k.encode(), to_mx(f))
        return s
    a = np.asarray(v, dtype=np.float64)
    if a.ndim < 2:
        a = a.reshape(1, -1) if a.ndim == 1 else a.reshape(1, 1)
    dims = (ctypes.c_longlong * a.ndim)(*a.shape)
    buf = np.asfortranarray(a)
    return L.mxhost_double(a.ndim, dims, buf.ctypes.data_as(ctypes.c_void_p))


def from_mx(p):
    L = mx()
    dims = (ctypes.c_longlong * 8)()
    nd = L.mxhost_dims(p, dims)
    shape = tuple(dims[k] for k in range(nd))
    n = int(np.prod(shape))
    if n == 0:
        return np.zeros(shape, order="F")
    buf = (ctypes.c_double * n).from_address(L.mxGetPr(p))
    return np.array(np.frombuffer(buf, dtype=np.float64).reshape(shape, order="F"), order="F")


class MexError(RuntimeError):
    pass


def call(name, nout, *args):
    """[out1, ..., outN] = name(args...) through mexFunction; raises MexError
    with the gateway's mexErrMsgIdAndTxt message."""
    L = mx()
    fn = gateway(name)
    pin = (ctypes.c_void_p * max(len(args), 1))(*[to_mx(a) for a in args])
    pout = (ctypes.c_void_p * max(nout, 1))()
    err = ctypes.create_string_buffer(512)
    rc = L.mxhost_call(fn, nout, pout, len(args), pin, err, 512)
    for k in range(len(args)):
        L.mxDestroyArray(pin[k])
    if rc:
        raise MexError(err.value.decode())
    outs = []
    for k in range(max(nout, 1)):
        if pout[k]:
            outs.append(from_mx(pout[k]))
            L.mxDestroyArray(pout[k])
    return outs
