"""ctypes binding of libpoissbox_gpu.so (the C ABI declared in include/poissbox_gpu.h).

The shared library is built in-tree (poissbox_amd/libpoissbox_gpu.so, see csrc/Makefile). There is
no CPU fallback: if the library is missing or cannot be loaded, importing the API raises.
"""
import ctypes as C
import os
import subprocess

_HERE = os.path.dirname(os.path.abspath(__file__))
# PB_LIB: load an alternative build of the same ABI (kernel-variant experiments, scripts/)
LIB_PATH = os.environ.get("PB_LIB") or os.path.join(_HERE, "libpoissbox_gpu.so")

c_i64 = C.c_int64
c_d = C.c_double
c_p = C.c_void_p
P_d = C.POINTER(C.c_double)
P_i64 = C.POINTER(C.c_int64)


class PbError(RuntimeError):
    def __init__(self, code, msg, where):
        super().__init__(f"{where} failed (code {code}): {msg}")
        self.code = code


class KspOpts(C.Structure):
    _fields_ = [("rtol", c_d), ("atol", c_d), ("dtol", c_d), ("max_it", c_i64),
                ("ksp_type", C.c_int), ("pc_type", C.c_int), ("nullspace", C.c_int),
                ("monitor", C.c_int), ("converged_reason", C.c_int), ("check_every", C.c_int),
                ("mg_levels", C.c_int), ("mg_coarse_its", C.c_int), ("sor_omega", c_d),
                ("cg_single_reduction", C.c_int)]


class KspResult(C.Structure):
    _fields_ = [("reason", C.c_int), ("its", c_i64), ("rnorm", c_d), ("rnorm0", c_d),
                ("nhist", c_i64)]


SENDRECV_FN = C.CFUNCTYPE(C.c_int, c_p, P_d, P_d, P_d, P_d, c_i64)
ALLREDUCE_FN = C.CFUNCTYPE(C.c_int, c_p, P_d, C.c_int)
ALLTOALLV_FN = C.CFUNCTYPE(C.c_int, c_p, P_d, P_i64, P_d, P_i64)

# name -> argtypes (all functions return int error codes unless listed in _RESTYPES)
_SIGS = {
    "pb_last_error": [],
    "pb_version": [C.POINTER(C.c_int), C.POINTER(C.c_int)],
    "pb_lapl_1d_coeffs": [c_d, P_d],
    "pb_lapl_star_coeffs": [c_d, c_d, c_d, P_d],
    "pb_comm_unique_id": [C.c_char_p],
    "pb_ctx_create": [C.c_int, C.c_int, C.c_int, C.c_char_p, C.POINTER(c_p)],
    "pb_ctx_set_host_transport": [c_p, SENDRECV_FN, ALLREDUCE_FN, c_p],
    "pb_ctx_set_host_alltoallv": [c_p, ALLTOALLV_FN, c_p],
    "pb_ctx_get_rank": [c_p, C.POINTER(C.c_int), C.POINTER(C.c_int)],
    "pb_ctx_sync": [c_p],
    "pb_ctx_barrier": [c_p],
    "pb_ctx_comm_status": [c_p, C.POINTER(C.c_int)],
    "pb_ctx_comm_info": [c_p, C.POINTER(C.c_int), C.POINTER(C.c_int), C.POINTER(C.c_int)],
    "pb_ctx_create_from_env": [C.c_int, C.POINTER(c_p)],
    "pb_ctx_allreduce_host": [c_p, P_d, C.c_int],
    "pb_ctx_destroy": [c_p],
    "pb_ctx_set_timing": [c_p, C.c_int],
    "pb_ctx_set_timing_filter": [c_p, C.c_int, C.c_char_p, C.c_int],
    "pb_tune_set": [C.c_char_p, C.c_int],
    "pb_tune_get": [C.c_char_p, C.POINTER(C.c_int), C.POINTER(C.c_int)],
    "pb_tune_reset": [],
    "pb_ctx_get_timing": [c_p, C.c_char_p, P_d, P_i64],
    "pb_ctx_get_timing_samples": [c_p, C.c_char_p, C.POINTER(C.c_float), c_i64, P_i64],
    "pb_ctx_reset_timing": [c_p],
    "pb_ctx_copy_probe": [c_p, c_i64, C.c_int, P_d, P_d],
    "pb_vec_copy_probe": [c_p, c_p, C.c_int, P_d, P_d],
    "pb_slab_partition": [c_i64, C.c_int, C.c_int, P_i64, P_i64],
    "pb_grid_create": [c_p, P_i64, P_d, C.POINTER(c_p)],
    "pb_grid_get_corners": [c_p, P_i64, P_i64],
    "pb_grid_get_info": [c_p, P_i64, P_d, P_i64],
    "pb_grid_destroy": [c_p],
    "pb_vec_create": [c_p, C.POINTER(c_p)],
    "pb_vec_duplicate": [c_p, C.POINTER(c_p)],
    "pb_vec_destroy": [c_p],
    "pb_vec_set": [c_p, c_d],
    "pb_vec_copy": [c_p, c_p],
    "pb_vec_axpy": [c_p, c_d, c_p],
    "pb_vec_aypx": [c_p, c_d, c_p],
    "pb_vec_scale": [c_p, c_d],
    "pb_vec_dot": [c_p, c_p, P_d],
    "pb_vec_norm2": [c_p, P_d],
    "pb_vec_sum": [c_p, P_d],
    "pb_vec_set_values_host": [c_p, P_d],
    "pb_vec_get_values_host": [c_p, P_d],
    "pb_vec_set_random": [c_p, C.c_uint64],
    "pb_vec_device_ptr": [c_p, C.POINTER(c_p), P_i64],
    "pb_op_create": [c_p, C.c_int, P_d, C.POINTER(c_p)],
    "pb_op_apply": [c_p, c_p, c_p],
    "pb_op_set_deltas": [c_p, P_d],
    "pb_op_get_diagonal": [c_p, P_d],
    "pb_op_destroy": [c_p],
    "pb_op_get_ownership_range": [c_p, P_i64, P_i64],
    "pb_vec_get_ownership_range": [c_p, P_i64, P_i64],
    "pb_ksp_opts_default": [C.POINTER(KspOpts)],
    "pb_ksp_opts_parse": [C.POINTER(KspOpts), C.c_int, C.POINTER(C.c_char_p)],
    "pb_ksp_create": [c_p, c_p, C.POINTER(KspOpts), C.POINTER(c_p)],
    "pb_ksp_solve": [c_p, c_p, c_p, C.POINTER(KspResult), P_d, c_i64],
    "pb_ksp_begin": [c_p, c_p, c_p],
    "pb_ksp_iterate": [c_p, c_i64],
    "pb_ksp_end": [c_p, C.POINTER(KspResult), P_d, c_i64],
    "pb_ksp_destroy": [c_p],
    "pb_ksp_pc_apply": [c_p, c_p, c_p],
    "pb_ksp_pc_levels": [c_p, C.POINTER(C.c_int)],
    "pb_solve": [c_p, c_p, C.POINTER(KspOpts), c_p, c_p, C.POINTER(KspResult), P_d, c_i64],
    "pb_tdma_batched": [c_p, c_i64, c_i64, c_i64, c_i64, c_p, c_p, c_p, c_p, C.c_int],
    "pb_pcr_alpha_batched": [c_p, c_i64, c_i64, c_i64, c_i64, c_d, c_p],
    "pb_compact_grad": [c_p, P_d, c_p, C.POINTER(c_p)],
    "pb_compact_div": [c_p, P_d, C.POINTER(c_p), c_p],
    "pb_compact_interp": [c_p, C.c_int, c_p, c_p],
    "pb_compact_lapl": [c_p, P_d, c_p, c_p],
    "pb_compact_lapl_fast": [c_p, P_d, c_p, c_p],
    "pb_compact_1d_batched": [c_p, C.c_int, C.c_int, c_d, c_i64, c_i64, c_i64, c_i64, c_p, c_p],
    "pb_tdma_sweeps_batched": [c_p, c_i64, c_i64, c_i64, c_i64, c_p, c_p, c_p, c_p, C.c_int],
    "pb_tdma_sweeps_batched_host": [c_p, c_i64, c_i64, c_i64, c_i64, P_d, P_d, P_d, P_d,
                                    C.c_int],
    "pb_tdma_batched_host": [c_p, c_i64, c_i64, c_i64, c_i64, P_d, P_d, P_d, P_d, C.c_int],
    "pb_compact_1d_batched_host": [c_p, C.c_int, C.c_int, c_d, c_i64, c_i64, c_i64, c_i64, P_d,
                                   P_d],
    "pb_compact_grad_host": [c_p, P_i64, P_d, P_d, P_d],
    "pb_compact_div_host": [c_p, P_i64, P_d, P_d, P_d],
    "pb_compact_interp_host": [c_p, P_i64, C.c_int, P_d, P_d],
    "pb_compact_lapl_host": [c_p, P_i64, P_d, P_d, P_d],
}
_RESTYPES = {"pb_last_error": C.c_char_p}

EXPORTED = tuple(_SIGS)

_lib = None


def build():
    """Compile libpoissbox_gpu.so for gfx950 (hipcc cross-compiles without a GPU)."""
    subprocess.run(["make", "-s", "-j8", "-C", os.path.join(_HERE, "csrc")], check=True)


def load():
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise ImportError(f"{LIB_PATH} not built: run `make -C poissbox_amd/csrc` "
                          "(no CPU fallback exists)")
    lib = C.CDLL(LIB_PATH)
    for name, argtypes in _SIGS.items():
        fn = getattr(lib, name)
        fn.argtypes = argtypes
        fn.restype = _RESTYPES.get(name, C.c_int)
    _lib = lib
    return lib


def call(name, *args):
    lib = load()
    rc = getattr(lib, name)(*args)
    if rc != 0:
        raise PbError(rc, lib.pb_last_error().decode(errors="replace"), name)
    return rc
