"""TEST INFRASTRUCTURE: drive the MEX gateway (colaborativempc-_amd/mex/cmpc_quadprog_mex.c)
through the mock mex.h build (libcmpc_mex_mock.so) — MATLAB is not available here."""
import ctypes as ct
import os

import numpy as np

from cmpc import _lib as L

MOCK = os.path.join(os.path.dirname(L.LIB_PATH), "libcmpc_mex_mock.so")
LPV_MOCK = os.path.join(os.path.dirname(L.LIB_PATH), "libcmpc_lpv_mex_mock.so")
_M = {}


def lib(path=MOCK):
    """The mock-MEX build of a gateway: cmpc_quadprog (default) or cmpc_lpv (LPV_MOCK).  Arrays made
    by either build's mock_* helpers are interchangeable (same mock mxArray)."""
    if path not in _M:
        L.load()   # torch first, then libcmpc (one HIP runtime), then the gateway
        m = ct.CDLL(path)
        m.mock_array.restype = ct.c_void_p
        m.mock_array.argtypes = [ct.c_int, ct.POINTER(ct.c_long), ct.POINTER(ct.c_double)]
        m.mock_sparse.restype = ct.c_void_p
        m.mock_sparse.argtypes = [ct.c_long, ct.c_long, ct.c_long, ct.POINTER(ct.c_double), ct.POINTER(ct.c_long),
                                  ct.POINTER(ct.c_long)]
        m.mock_struct.restype = ct.c_void_p
        m.mock_struct.argtypes = [ct.c_int, ct.POINTER(ct.c_char_p), ct.POINTER(ct.c_void_p)]
        m.mock_struct2.restype = ct.c_void_p
        m.mock_struct2.argtypes = [ct.c_char_p, ct.c_void_p, ct.c_char_p, ct.c_void_p]
        m.mock_call.restype = ct.c_int
        m.mock_call.argtypes = [ct.c_int, ct.POINTER(ct.c_void_p), ct.c_int, ct.POINTER(ct.c_void_p)]
        m.mock_err_id.restype = ct.c_char_p
        m.mock_err_msg.restype = ct.c_char_p
        m.mock_data.restype = ct.POINTER(ct.c_double)
        m.mock_data.argtypes = [ct.c_void_p]
        m.mock_numel.restype = ct.c_size_t
        m.mock_numel.argtypes = [ct.c_void_p]
        m.mock_field.restype = ct.c_void_p
        m.mock_field.argtypes = [ct.c_void_p, ct.c_char_p]
        m.mock_string.restype = ct.c_char_p
        m.mock_string.argtypes = [ct.c_void_p]
        m.mxCreateString.restype = ct.c_void_p
        m.mxCreateString.argtypes = [ct.c_char_p]
        _M[path] = m
    return _M[path]


def mx_str(s):
    """A MATLAB char array (command strings of cmpc_lpv)."""
    return lib().mxCreateString(s.encode())


def call_lpv(ps, nlhs):
    """cmpc_lpv(...) on prepared mxArray pointers -> (outputs | None, (err_id, err_msg) | None)."""
    m = lib(LPV_MOCK)
    prhs = (ct.c_void_p * len(ps))(*ps)
    plhs = (ct.c_void_p * nlhs)()
    rc = m.mock_call(nlhs, plhs, len(ps), prhs)
    if rc:
        return None, (m.mock_err_id().decode(), m.mock_err_msg().decode())
    return list(plhs), None


def mx(a):
    """numpy array -> mock mxArray (MATLAB column-major; 1-D becomes a column; None -> [])."""
    m = lib()
    if a is None:
        dims = (ct.c_long * 2)(0, 0)
        return m.mock_array(2, dims, None)
    a = np.asarray(a, dtype=np.float64)
    if a.ndim == 1:
        a = a[:, None]
    dims = (ct.c_long * a.ndim)(*a.shape)
    buf = np.asfortranarray(a).ravel(order="F")
    return m.mock_array(a.ndim, dims, buf.ctypes.data_as(ct.POINTER(ct.c_double)))


def mx_sparse(a):
    """scipy sparse / dense 2-D -> mock sparse mxArray (CSC, as MATLAB stores it)."""
    import scipy.sparse as sp

    m = lib()
    c = sp.csc_matrix(a)
    c.sort_indices()
    pr = np.ascontiguousarray(c.data, dtype=np.float64)
    ir = np.ascontiguousarray(c.indices, dtype=np.int64)
    jc = np.ascontiguousarray(c.indptr, dtype=np.int64)
    return m.mock_sparse(c.shape[0], c.shape[1], c.nnz, pr.ctypes.data_as(ct.POINTER(ct.c_double)),
                         ir.ctypes.data_as(ct.POINTER(ct.c_long)), jc.ctypes.data_as(ct.POINTER(ct.c_long)))


def mx_struct(fields):
    """dict name -> numpy array (or an mxArray pointer from mx/mx_sparse) -> 1 x 1 struct."""
    m = lib()
    names = (ct.c_char_p * len(fields))(*[k.encode() for k in fields])
    vals = (ct.c_void_p * len(fields))(*[v if isinstance(v, int) else mx(v) for v in fields.values()])
    return m.mock_struct(len(fields), names, vals)


def call_raw(ps, nlhs):
    """mexFunction on prepared mxArray pointers -> (outputs | None, (err_id, err_msg) | None)."""
    m = lib()
    prhs = (ct.c_void_p * len(ps))(*ps)
    plhs = (ct.c_void_p * nlhs)()
    rc = m.mock_call(nlhs, plhs, len(ps), prhs)
    if rc:
        return None, (m.mock_err_id().decode(), m.mock_err_msg().decode())
    return list(plhs), None


def values(p):
    m = lib()
    k = m.mock_numel(p)
    return np.ctypeslib.as_array(m.mock_data(p), shape=(k,)).copy() if k else np.zeros(0)


def call(args, nlhs=5, opts=None):
    """cmpc_quadprog(*args [, x0=[], opts]) -> (outputs | None, (err_id, err_msg) | None)."""
    m = lib()
    ps = [mx(a) for a in args]
    if opts is not None:
        while len(ps) < 8:
            ps.append(mx(None))
        ps.append(mx(None))  # x0
        ps.append(m.mock_struct2(b"MaxIterations", mx(np.array([opts.get("MaxIterations", 0.0)])),
                                 b"OptimalityTolerance", mx(np.array([opts.get("OptimalityTolerance", 0.0)]))))
    prhs = (ct.c_void_p * len(ps))(*ps)
    plhs = (ct.c_void_p * nlhs)()
    rc = m.mock_call(nlhs, plhs, len(ps), prhs)
    if rc:
        return None, (m.mock_err_id().decode(), m.mock_err_msg().decode())
    return list(plhs), None


def field(p, name):
    return lib().mock_field(p, name.encode())
