"""ctypes binding of libmceik_hip.so (the C-ABI in include/*.h).

The HIP library IS the product: there is no CPU fallback.  If the library is
missing or cannot be loaded this module raises, loudly.
"""
import ctypes as C
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, "libmceik_hip.so")

_lib = None


class FsmBatch(C.Structure):
    """mceik_fsm_batch (include/mceik_eikonal.h)."""
    _fields_ = [("nx", C.c_int), ("ny", C.c_int), ("nz", C.c_int),
                ("h", C.c_double), ("x0", C.c_double), ("y0", C.c_double), ("z0", C.c_double),
                ("maxit", C.c_int), ("tol", C.c_double), ("precision", C.c_int),
                ("nmodel", C.c_int), ("nstat", C.c_int), ("nsrc", C.c_int),
                ("src", C.c_void_p), ("slow_mode", C.c_int), ("slow", C.c_void_p),
                ("nrx", C.c_int), ("nry", C.c_int), ("nrz", C.c_int),
                ("nev", C.c_int), ("ev_node", C.c_void_p), ("ttab", C.c_void_p),
                ("u_out", C.c_void_p), ("niter", C.c_void_p), ("ierr", C.c_void_p),
                ("max_sweeps", C.c_int), ("iter_total", C.c_void_p), ("fast_sqrt", C.c_int),
                ("visit_stats", C.c_void_p), ("solve_order", C.c_void_p), ("solve_clock", C.c_void_p),
                ("max_waves", C.c_int), ("traffic", C.c_void_p), ("step_z", C.c_int),
                ("ev_frac", C.c_void_p), ("model_phase", C.c_void_p), ("nphase", C.c_int),
                ("skip", C.c_void_p), ("solve_count", C.c_void_p)]


class RelocateBatch(C.Structure):
    """mceik_relocate_batch (include/mceik_eikonal.h)."""
    _fields_ = [("ldgrd", C.c_int), ("ngrd", C.c_int), ("nev", C.c_int), ("iwantOT", C.c_int),
                ("t0use", C.c_float), ("tables", C.c_void_p), ("ev_ptr", C.c_void_p), ("obs_row", C.c_void_p),
                ("tc", C.c_void_p), ("wt", C.c_void_p), ("xnorm", C.c_void_p), ("t0", C.c_void_p),
                ("out", C.c_void_p), ("log_pdf", C.c_int), ("nrows", C.c_int), ("nobs", C.c_int)]


class McmcParms(C.Structure):
    _fields_ = [("resdir", C.c_char * 512), ("nburnIn", C.c_int), ("niter", C.c_int), ("keepK", C.c_int)]


class EikParms(C.Structure):
    _fields_ = [("tol", C.c_double), ("maxit", C.c_int)]


class MceikParms(C.Structure):
    """struct mceik_parms_struct (include/mceik_struct.h; reference mceik_struct.h:68-90)."""
    _fields_ = [("mcparms", McmcParms), ("eikparms", EikParms), ("projnm", C.c_char * 128),
                ("scratch_dir", C.c_char * 512),
                ("x0", C.c_double), ("y0", C.c_double), ("z0", C.c_double),
                ("dx", C.c_double), ("dy", C.c_double), ("dz", C.c_double),
                ("ndivx", C.c_int), ("ndivy", C.c_int), ("ndivz", C.c_int),
                ("nrefx", C.c_int), ("nrefy", C.c_int), ("nrefz", C.c_int)]


class CatalogStruct(C.Structure):
    """struct mceik_catalog_struct (reference mceik_struct.h:10-32)."""
    _fields_ = [(n, C.POINTER(C.c_double)) for n in ("xsrc", "ysrc", "zsrc", "tori", "tobs", "test", "varObs")] + \
               [(n, C.POINTER(C.c_int)) for n in ("luseObs", "pickType", "statPtr", "obsPtr")] + \
               [("nevents", C.c_int)]


class StationsStruct(C.Structure):
    """struct mceik_stations_struct (reference mceik_struct.h:34-49)."""
    _fields_ = [(n, C.POINTER(C.c_char_p)) for n in ("netw", "stnm", "chan", "loc")] + \
               [(n, C.POINTER(C.c_double)) for n in ("xrec", "yrec", "zrec", "pcorr", "scorr")] + \
               [(n, C.POINTER(C.c_int)) for n in ("lhasP", "lhasS")] + \
               [("nstat", C.c_int), ("lcartesian", C.c_int)]


class McmcOpts(C.Structure):
    """mceik_mcmc_opts (include/mceik.h)."""
    _fields_ = [("nx", C.c_int), ("ny", C.c_int), ("nz", C.c_int), ("nchains", C.c_int),
                ("chain_offset", C.c_int), ("vmin", C.c_int), ("vmax", C.c_int), ("dvmax", C.c_int),
                ("seed", C.c_uint32), ("max_samples", C.c_int), ("device", C.c_int),
                ("precision", C.c_int), ("max_waves", C.c_int), ("tt_interp", C.c_int),
                ("nphase", C.c_int), ("vsmin", C.c_int), ("vsmax", C.c_int), ("mask_s", C.c_int)]


class McmcInfo(C.Structure):
    """mceik_mcmc_info (include/mceik.h)."""
    _fields_ = [("npipe", C.c_int), ("nphase", C.c_int), ("step_z", C.c_int), ("fixed_layout", C.c_int),
                ("chains", C.c_int * 4), ("waves", C.c_int * 4), ("workspace_bytes", C.c_size_t * 4),
                ("lds_bytes", C.c_size_t), ("masked_s", C.c_int), ("kernel", C.c_char * 64),
                ("multi_step", C.c_int)]


# every extern "C" symbol include/*.h declares
EXPORTS = ("eikonal3d_serial_driver", "eikonal3d_serial_driver_sp", "eikonal3d_batch_solve", "eikonal3d_initialize", "eikonal3d_solve",
           "eikonal3d_finalize", "locate3d_gridsearch__double64", "locate3d_gridsearch__float64",
           "locate_l2_gridSearch__double64",
           "locate_l2_gridSearch__float64", "mceik_relocate",
           "locate3d_initialize", "locate3d_gridsearch", "locate3d_finalize",
           "mceik_fsm_workspace_bytes", "mceik_fsm_batch_solve", "mceik_fsm_bytes_per_node_sweep", "mceik_fsm_step_z",
           "mceik_fsm_kernel_name", "mceik_fsm_lds_bytes",
           "mceik_memcpy",
           "mceik_mcmc_init", "mceik_mcmc_run", "mceik_mcmc_set_stream", "mceik_mcmc_sync",
           "mceik_mcmc_get_state", "mceik_mcmc_get_samples", "mceik_mcmc_last", "mceik_mcmc_fsm_stats",
           "mceik_mcmc_checkpoint", "mceik_mcmc_restore", "mceik_mcmc_finalize", "mceik_mcmc_last_phase",
           "mceik_mcmc_get_info", "mceik_mcmc_fsm_solves",
           "mceik_parms_defaults", "mceik_parms_set", "mceik_parms_read", "mceik_parms_args", "mceik_parms_write",
           "mceik_comm_available", "mceik_comm_unique_id", "mceik_comm_init", "mceik_comm_finalize", "mceik_mcmc_gather",
           "os_path_exists", "os_path_isdir", "os_path_isfile", "os_makedirs", "os_mkdir")


def lib():
    """Load libmceik_hip.so (raises OSError/ImportError if absent: no fallback)."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise ImportError(f"mceik_amd: HIP library {LIB_PATH} is missing; build it with "
                          f"`make -C {_HERE}` (or __graft_entry__.build()). No CPU fallback exists.")
    L = C.CDLL(LIB_PATH)
    pi = C.POINTER(C.c_int); pd = C.POINTER(C.c_double)
    for name in ("eikonal3d_serial_driver", "eikonal3d_serial_driver_sp"):
        f = getattr(L, name)
        f.restype = None
        f.argtypes = [pi] * 7 + [pd] * 5 + [C.c_void_p] * 6 + [pi]
    L.eikonal3d_initialize.restype = None
    L.eikonal3d_initialize.argtypes = [pi] * 10 + [pd] * 5 + [pi]
    L.eikonal3d_solve.restype = None
    L.eikonal3d_solve.argtypes = [pi] * 3 + [C.c_void_p] * 6 + [pi]
    L.eikonal3d_finalize.restype = None
    L.eikonal3d_finalize.argtypes = [pi, pi]
    for name in ("locate3d_gridsearch__double64", "locate3d_gridsearch__float64"):
        f = getattr(L, name)
        f.restype = None
        f.argtypes = [pi] * 4 + [C.c_void_p] * 5 + [pi]
    L.locate_l2_gridSearch__double64.restype = C.c_int
    L.locate_l2_gridSearch__double64.argtypes = [C.c_int] * 4 + [C.c_double] + [C.c_void_p] * 7
    L.eikonal3d_batch_solve.restype = C.c_int
    L.eikonal3d_batch_solve.argtypes = [C.c_int] * 5 + [C.c_double] * 4 + [C.c_int, C.c_double] + [C.c_void_p] * 5
    L.mceik_fsm_workspace_bytes.restype = C.c_size_t
    L.mceik_fsm_workspace_bytes.argtypes = [C.POINTER(FsmBatch)]
    L.mceik_fsm_step_z.restype = C.c_int
    L.mceik_fsm_step_z.argtypes = [C.POINTER(FsmBatch)]
    L.mceik_fsm_kernel_name.restype = C.c_char_p
    L.mceik_fsm_kernel_name.argtypes = [C.POINTER(FsmBatch)]
    L.mceik_fsm_lds_bytes.restype = C.c_size_t
    L.mceik_fsm_lds_bytes.argtypes = [C.POINTER(FsmBatch)]
    L.mceik_fsm_bytes_per_node_sweep.restype = C.c_double
    L.mceik_fsm_bytes_per_node_sweep.argtypes = [C.POINTER(FsmBatch)]
    L.mceik_fsm_batch_solve.restype = C.c_int
    L.mceik_fsm_batch_solve.argtypes = [C.POINTER(FsmBatch), C.c_void_p, C.c_size_t, C.c_void_p]
    L.mceik_memcpy.restype = C.c_int
    L.mceik_memcpy.argtypes = [C.c_void_p, C.c_void_p, C.c_size_t, C.c_int]
    L.locate_l2_gridSearch__float64.restype = C.c_int
    L.locate_l2_gridSearch__float64.argtypes = [C.c_int] * 4 + [C.c_float] + [C.c_void_p] * 7
    L.mceik_relocate.restype = C.c_int
    L.mceik_relocate.argtypes = [C.POINTER(RelocateBatch), C.c_void_p]
    L.mceik_mcmc_init.restype = C.c_int
    L.mceik_mcmc_init.argtypes = [C.POINTER(MceikParms), C.POINTER(StationsStruct), C.POINTER(CatalogStruct),
                                  C.POINTER(McmcOpts), C.c_void_p, C.POINTER(C.c_void_p)]
    L.mceik_mcmc_run.restype = C.c_int
    L.mceik_mcmc_run.argtypes = [C.c_void_p, C.c_int]
    L.mceik_mcmc_set_stream.restype = C.c_int
    L.mceik_mcmc_set_stream.argtypes = [C.c_void_p, C.c_void_p]
    L.mceik_mcmc_sync.restype = C.c_int
    L.mceik_mcmc_sync.argtypes = [C.c_void_p]
    L.mceik_mcmc_get_state.restype = C.c_int
    L.mceik_mcmc_get_state.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, C.POINTER(C.c_longlong)]
    L.mceik_mcmc_get_samples.restype = C.c_int
    L.mceik_mcmc_get_samples.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p, C.c_int, C.c_int, pi]
    L.mceik_mcmc_last.restype = C.c_int
    L.mceik_mcmc_last.argtypes = [C.c_void_p] + [C.POINTER(C.c_void_p)] * 4
    L.mceik_mcmc_checkpoint.restype = C.c_int
    L.mceik_mcmc_checkpoint.argtypes = [C.c_void_p] + [C.c_void_p] * 3 + [C.POINTER(C.c_longlong), pi]
    L.mceik_mcmc_restore.restype = C.c_int
    L.mceik_mcmc_restore.argtypes = [C.c_void_p] + [C.c_void_p] * 3 + [C.c_longlong, C.c_int]
    L.mceik_mcmc_fsm_stats.restype = C.c_int
    L.mceik_mcmc_fsm_stats.argtypes = [C.c_void_p, C.POINTER(C.c_double), C.POINTER(C.c_longlong),
                                       C.POINTER(C.c_ulonglong), C.POINTER(C.c_ulonglong), C.c_int]
    L.mceik_mcmc_fsm_solves.restype = C.c_int
    L.mceik_mcmc_fsm_solves.argtypes = [C.c_void_p, C.POINTER(C.c_ulonglong)]
    L.mceik_comm_available.restype = C.c_int
    L.mceik_comm_available.argtypes = []
    L.mceik_comm_unique_id.restype = C.c_int
    L.mceik_comm_unique_id.argtypes = [C.c_void_p]
    L.mceik_comm_init.restype = C.c_int
    L.mceik_comm_init.argtypes = [C.c_void_p, C.c_int, C.c_int, C.c_int, C.POINTER(C.c_void_p)]
    L.mceik_comm_finalize.restype = C.c_int
    L.mceik_comm_finalize.argtypes = [C.POINTER(C.c_void_p)]
    L.mceik_mcmc_gather.restype = C.c_int
    L.mceik_mcmc_gather.argtypes = [C.c_void_p, C.c_void_p, C.c_int, C.c_int, C.c_int, C.c_void_p, C.c_void_p]
    L.mceik_mcmc_last_phase.restype = C.c_int
    L.mceik_mcmc_last_phase.argtypes = [C.c_void_p, C.POINTER(C.c_void_p)]
    L.mceik_mcmc_get_info.restype = C.c_int
    L.mceik_mcmc_get_info.argtypes = [C.c_void_p, C.POINTER(McmcInfo)]
    L.mceik_mcmc_finalize.restype = C.c_int
    L.mceik_mcmc_finalize.argtypes = [C.POINTER(C.c_void_p)]
    _lib = L
    return L
