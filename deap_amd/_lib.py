"""ctypes binding of ``libdeapmi.so`` (the C ABI declared in ``include/deapmi.h``).

This is the only place the Python host layer touches native code.  The library
is built in-tree (``deap_amd/libdeapmi.so``) by ``deap_amd/csrc/Makefile``;
there is no CPU fallback: if the library is missing every device operation
raises :class:`DeviceUnavailable`.

Error mapping follows the reference's exception types:
``DM_ERR_INVALID`` -> ValueError, ``DM_ERR_INDEX`` -> IndexError (short
mu/sigma sequences, ``deap/tools/mutation.py:37-42``), anything else ->
RuntimeError.
"""
import ctypes
import os
import threading

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("DEAPMI_LIB") or os.path.join(_HERE, "libdeapmi.so")

DM_OK, DM_ERR_INVALID, DM_ERR_INDEX, DM_ERR_HIP, DM_ERR_NOMEM, DM_ERR_UNSUPPORTED = range(6)
DM_BITS, DM_F32, DM_F64 = 0, 1, 2
DM_CX_NONE, DM_CX_TWOPOINT, DM_CX_BLEND = 0, 1, 2
DM_MUT_NONE, DM_MUT_FLIPBIT, DM_MUT_GAUSSIAN = 0, 1, 2
DM_SEL_IDENTITY, DM_SEL_INDEX, DM_SEL_TOURNAMENT, DM_SEL_RANDOM = 0, 1, 2, 3
DM_RNG_NATIVE, DM_RNG_INJECT, DM_RNG_DUMP = 0, 1, 2
DM_TIME_GENERATION, DM_TIME_DOMINANCE, DM_TIME_PEEL, DM_TIME_PEEL_CHAIN = 0, 1, 2, 3
# enum dm_dom_path: sortNondominated's default path and its cross-check paths
DM_DOM_PATHS = {"default": 0, "compare": 1, "peel_d": 2, "ballot": 3, "lds": 4}
(DM_EVAL_NONE, DM_EVAL_ONEMAX, DM_EVAL_RASTRIGIN, DM_EVAL_ROSENBROCK, DM_EVAL_ZDT1,
 DM_EVAL_ZDT2, DM_EVAL_ZDT3, DM_EVAL_ZDT4, DM_EVAL_ZDT6, DM_EVAL_DTLZ1, DM_EVAL_DTLZ2,
 DM_EVAL_DTLZ3, DM_EVAL_DTLZ4, DM_EVAL_SPHERE) = range(14)
DM_MAX_OBJ = 8

_p = ctypes.c_void_p
_i32 = ctypes.c_int32
_i64 = ctypes.c_int64
_u32 = ctypes.c_uint32
_u64 = ctypes.c_uint64
_f64 = ctypes.c_double


class DevicePop(ctypes.Structure):
    """struct dm_pop"""
    _fields_ = [("genes", _p), ("wvalues", _p), ("valid", _p), ("n", _i64), ("stride", _i64),
                ("dim", _i32), ("gtype", _i32), ("nobj", _i32), ("reserved", _i32)]


class Eval(ctypes.Structure):
    """struct dm_eval"""
    _fields_ = [("fn", _i32), ("obj", _i32), ("alpha", _f64), ("weights", _f64 * DM_MAX_OBJ)]


class Variation(ctypes.Structure):
    """struct dm_variation"""
    _fields_ = [("cx", _i32), ("mut", _i32), ("cxpb", _f64), ("mutpb", _f64), ("alpha", _f64),
                ("indpb", _f64), ("mu", _f64), ("sigma", _f64), ("mu_vec", _p),
                ("sigma_vec", _p)]


class Rng(ctypes.Structure):
    """struct dm_rng"""
    _fields_ = [("seed", _u64), ("island", _u32), ("gen", _u32)]


class Decisions(ctypes.Structure):
    """struct dm_decisions"""
    _fields_ = [("aspirants", _p), ("cx_flag", _p), ("cx_raw", _p), ("blend_u", _p),
                ("mut_flag", _p), ("mut_mask", _p), ("gauss", _p), ("varor_op", _p),
                ("varor_idx", _p)]


class BoundedVar(ctypes.Structure):
    """struct dm_bounded_var"""
    _fields_ = [("cx", _i32), ("mut", _i32), ("cxpb", _f64), ("eta_cx", _f64), ("eta_mut", _f64),
                ("indpb", _f64), ("low", _f64), ("up", _f64), ("low_vec", _p), ("up_vec", _p)]


# name -> (restype, argtypes); mirrors include/deapmi.h one to one.
_PP = ctypes.POINTER
SIGNATURES = {
    "dm_last_error": (ctypes.c_char_p, []),
    "dm_version": (ctypes.c_char_p, []),
    "dm_ctx_create": (ctypes.c_int, [ctypes.c_int, _p, _PP(_p)]),
    "dm_ctx_destroy": (ctypes.c_int, [_p]),
    "dm_ctx_set_stream": (ctypes.c_int, [_p, _p]),
    "dm_ctx_sync": (ctypes.c_int, [_p]),
    "dm_zero": (ctypes.c_int, [_p, _p, _i64]),
    "dm_set_fitness": (ctypes.c_int, [_p, _p, _p, _i64, _p]),
    "dm_ctx_set_timing": (ctypes.c_int, [_p, _i32]),
    "dm_ctx_kernel_times": (ctypes.c_int, [_p, _p, _i32, _PP(_i32)]),
    "dm_ctx_set_timing_target": (ctypes.c_int, [_p, _i32]),
    "dm_ctx_set_dom_path": (ctypes.c_int, [_p, _i32]),
    "dm_ctx_dom_bitset": (ctypes.c_int, [_p, _i32]),
    "dm_ctx_reload_knobs": (ctypes.c_int, [_p]),
    "dm_philox_blocks": (ctypes.c_int, [_p, _PP(_u32), _PP(_u32), _i64, _p]),
    "dm_init_uniform": (ctypes.c_int, [_p, _PP(DevicePop), _f64, _f64, Rng]),
    "dm_evaluate": (ctypes.c_int, [_p, _PP(DevicePop), _PP(Eval), ctypes.c_int, _p]),
    "dm_sel_tournament": (ctypes.c_int, [_p, _PP(DevicePop), _i64, _i32, Rng, _i32,
                                         _PP(Decisions), _p]),
    "dm_sel_random": (ctypes.c_int, [_p, _i64, _i64, Rng, _i32, _PP(Decisions), _p]),
    "dm_sel_best": (ctypes.c_int, [_p, _PP(DevicePop), _i64, _p]),
    "dm_sel_worst": (ctypes.c_int, [_p, _PP(DevicePop), _i64, _p]),
    "dm_gather": (ctypes.c_int, [_p, _PP(DevicePop), _p, _PP(DevicePop)]),
    "dm_generation": (ctypes.c_int, [_p, _PP(DevicePop), _PP(DevicePop), _i32, _i32, _p,
                                     _PP(Variation), _PP(Eval), Rng, _i32, _PP(Decisions), _p]),
    "dm_var_or": (ctypes.c_int, [_p, _PP(DevicePop), _PP(DevicePop), _PP(Variation), _PP(Eval),
                                 Rng, _i32, _PP(Decisions), _p]),
    "dm_sort_nondominated": (ctypes.c_int, [_p, _PP(DevicePop), _i64, _i32, _p, _p, _p,
                                            _PP(_i64), _PP(_i32)]),
    "dm_crowding_dist": (ctypes.c_int, [_p, _PP(DevicePop), _PP(_f64), _p, _p, _i32, _p]),
    "dm_sel_nsga2": (ctypes.c_int, [_p, _PP(DevicePop), _PP(_f64), _i64, _p, _p]),
    "dm_sort_log_nondominated": (ctypes.c_int, [_p, _PP(DevicePop), _i64, _i32, _p, _p,
                                                _PP(_i64), _PP(_i32)]),
    "dm_sel_nsga2_log": (ctypes.c_int, [_p, _PP(DevicePop), _PP(_f64), _i64, _p, _p]),
    "dm_gather_f64": (ctypes.c_int, [_p, _p, _p, _i64, _p]),
    "dm_sel_tournament_dcd": (ctypes.c_int, [_p, _PP(DevicePop), _p, _i64, Rng, _i32, _p, _p, _p,
                                             _p]),
    "dm_vary_bounded": (ctypes.c_int, [_p, _PP(DevicePop), _p, _PP(DevicePop), _PP(BoundedVar),
                                       Rng, _i32, _p, _p, _p]),
    "dm_pack_rows": (ctypes.c_int, [_p, _PP(DevicePop), _p, _i64, _p]),
    "dm_pack_bytes": (_i64, [_PP(DevicePop), _i64]),
    "dm_mig_place": (ctypes.c_int, [_p, _PP(DevicePop), _p, _p, _i64, _p]),
    "dm_fitness_stats": (ctypes.c_int, [_p, _PP(DevicePop), _PP(_f64), _p]),
    "dm_sel_sample": (ctypes.c_int, [_p, _i64, _i64, Rng, _p]),
    "dm_mig_plan": (ctypes.c_int, [_i32, _PP(_i32), _PP(_i32), _i32, _i32, _p, _i32,
                                   _PP(_i32)]),
    "dm_mig_ring": (ctypes.c_int, [_p, _i32, _PP(DevicePop), _PP(_i32), _i64, _PP(_p), _PP(_p),
                                   _PP(_p)]),
    "dm_comm_get_unique_id": (ctypes.c_int, [_p]),
    "dm_comm_init": (ctypes.c_int, [_p, _i32, _i32, _p, _PP(_p)]),
    "dm_comm_destroy": (ctypes.c_int, [_p]),
    "dm_mig_ring_rccl": (ctypes.c_int, [_p, _p, _i32, _PP(DevicePop), _PP(_i32), _i32, _PP(_i32),
                                        _PP(_i32), _i64, _PP(_p), _PP(_p), _PP(_p), _i32]),
}

DM_HOP_LOCAL, DM_HOP_SEND, DM_HOP_RECV = 0, 1, 2
DM_MIG_FORCE_P2P = 1
DM_COMM_ID_BYTES = 128


class MigHop(ctypes.Structure):
    """struct dm_mig_hop"""
    _fields_ = [("kind", _i32), ("from_", _i32), ("to", _i32), ("peer", _i32)]


class DeviceUnavailable(RuntimeError):
    """Raised when the native library or a GPU is not available."""


_lib = None
_lib_err = None
_lock = threading.Lock()


def load(path=None):
    """Load (once) and return the CDLL with every exported signature bound."""
    global _lib, _lib_err
    with _lock:
        if _lib is not None:
            return _lib
        p = path or LIB_PATH
        if not os.path.exists(p):
            _lib_err = ("libdeapmi.so not built (%s); run `python -c 'import __graft_entry__ as g;"
                        " g.build()'` or `make -C deap_amd/csrc`" % p)
            raise DeviceUnavailable(_lib_err)
        lib = ctypes.CDLL(p)
        for name, (res, args) in SIGNATURES.items():
            fn = getattr(lib, name)
            fn.restype = res
            fn.argtypes = args
        _lib = lib
        return lib


def last_error():
    return load().dm_last_error().decode(errors="replace")


def check(rc, what=""):
    """Map a C status to the reference's Python exception types."""
    if rc == DM_OK:
        return
    msg = last_error()
    if what:
        msg = "%s: %s" % (what, msg)
    if rc == DM_ERR_INVALID:
        raise ValueError(msg)
    if rc == DM_ERR_INDEX:
        raise IndexError(msg)
    raise RuntimeError(msg)


def call(name, *args):
    """Invoke C entry point `name` and raise on a non-zero status."""
    fn = getattr(load(), name)
    check(fn(*args), name)
