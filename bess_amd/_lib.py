"""ctypes binding of libbessgpu.so (include/bessgpu.h).

The HIP library is the product: if it is missing this module raises instead of
falling back to anything else.
"""
import atexit
import ctypes as C
import os

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "libbessgpu.so")

BG_MAX_GATES = 8192
BG_DROP_GATE = 8192
BG_GATE_NONE = 0xFFFF
BG_CK_IP = 1
BG_CK_L4 = 2
BG_PATH_FORCE_LDS = 1
BG_PATH_NO_LDS = 2
BG_PATH_NO_SLAB = 4
BG_PATH_WM_NO_TAGS = 8
BG_PATH_ACL_SCAN = 16
BG_PATH_ACL_BV = 32
BG_PATH_ACL_LDS = 64
BG_PATH_LPM_DIR24 = 128
BG_PATH_PIPE_NO_RING = 256
BG_PATH_WM_NO_JIT = 512
BG_PATH_RING_HOST_DESC = 1024
KEY_BYTES = 64


class BessGpuError(RuntimeError):
    """A failing bg_* call: errno + the reference-style message."""

    def __init__(self, code, msg):
        super().__init__("[errno %d] %s" % (code, msg))
        self.code = code
        self.msg = msg


class bg_ctx(C.Structure):
    """a ProcessBatch's Context (core/module.h:59-75): current_ns,
    current_igate, the device of the call (-1: the module's), wid"""
    _fields_ = [("now_ns", C.c_uint64), ("igate", C.c_uint16),
                ("device", C.c_int16), ("wid", C.c_uint32)]


def make_ctx(igate=0, now=None, device=-1, wid=0):
    """a bg_ctx pointer argument; now None = the library's monotonic clock
    (then the whole ctx is NULL when igate and device are defaults too)"""
    if now is None and igate == 0 and device == -1 and wid == 0:
        return None
    if now is None:
        import time
        now = time.monotonic_ns()
    return C.byref(bg_ctx(int(now), int(igate), int(device), int(wid)))


class bg_field(C.Structure):
    _fields_ = [("offset", C.c_int32), ("size", C.c_int32), ("pos", C.c_int32),
                ("attr_id", C.c_int32), ("mask", C.c_uint64)]


_vp, _sz, _u16, _i32, _int = C.c_void_p, C.c_size_t, C.c_uint16, C.c_int32, C.c_int
_SIGS = {
    "bg_version": (C.c_char_p, []),
    "bg_last_error": (C.c_char_p, []),
    "bg_device_count": (_int, []),
    "bg_malloc": (_int, [_int, _sz, C.POINTER(_vp)]),
    "bg_free": (_int, [_vp]),
    "bg_memcpy_h2d": (_int, [_vp, _vp, _sz, _vp]),
    "bg_memcpy_d2h": (_int, [_vp, _vp, _sz, _vp]),
    "bg_stream_sync": (_int, [_vp]),
    "bg_em_create": (_int, [C.POINTER(bg_field), _int, C.POINTER(_vp)]),
    "bg_em_destroy": (None, [_vp]),
    "bg_em_key_size": (_sz, [_vp]),
    "bg_em_add": (_int, [_vp, _vp, _u16]),
    "bg_em_delete": (_int, [_vp, _vp]),
    "bg_em_clear": (None, [_vp]),
    "bg_em_count": (_sz, [_vp]),
    "bg_em_iter": (_int, [_vp, C.POINTER(_sz), _vp, C.POINTER(_u16)]),
    "bg_em_sync": (_int, [_vp, _int, _vp]),
    "bg_em_classify": (_int, [_vp, _vp, _sz, _sz, _u16, _vp, _vp]),
    "bg_em_process_host": (_int, [_vp, _vp, _sz, _u16, _vp, _vp]),
    "bg_em_plan": (_int, [_vp, _int, C.POINTER(C.c_uint64)]),
    "bg_em_add_many": (_int, [_vp, _vp, _sz, _sz, _vp, _int, _int]),
    "bg_em_part_count": (_int, [_vp, _int, _int, C.POINTER(C.c_uint64)]),
    "bg_em_plan_count": (_int, [_vp, _int, C.c_uint64, C.POINTER(C.c_uint64)]),
    "bg_em_build_part": (_int, [_vp, _int, _vp]),
    "bg_em_attach": (_int, [_vp, _int, _vp]),
    "bg_em_table_info": (_int, [_vp, C.POINTER(C.c_uint64), C.POINTER(_int)]),
    "bg_comm_unique_id": (_int, [_vp]),
    "bg_comm_init_rank": (_int, [_vp, _int, _int, _int, C.POINTER(_vp)]),
    "bg_comm_init_all": (_int, [_vp, _int, _vp]),
    "bg_comm_destroy": (None, [_vp]),
    "bg_comm_info": (_int, [_vp, C.POINTER(_int), C.POINTER(_int), C.POINTER(_int)]),
    "bg_em_allgather": (_int, [_vp, _vp, _vp]),
    "bg_comm_last_stats": (_int, [_vp, _vp, C.POINTER(C.c_uint64)]),
    "bg_em_allgather_all": (_int, [_vp, _vp, _int]),
    "bg_wm_create": (_int, [C.POINTER(bg_field), _int, C.POINTER(_vp)]),
    "bg_wm_destroy": (None, [_vp]),
    "bg_wm_key_size": (_sz, [_vp]),
    "bg_wm_add": (_int, [_vp, _vp, _vp, _i32, _u16]),
    "bg_wm_delete": (_int, [_vp, _vp, _vp]),
    "bg_wm_clear": (None, [_vp]),
    "bg_wm_num_tuples": (_int, [_vp]),
    "bg_wm_tuple_mask": (_int, [_vp, _int, _vp]),
    "bg_wm_tuple_count": (_sz, [_vp, _int]),
    "bg_wm_iter": (_int, [_vp, _int, C.POINTER(_sz), _vp, C.POINTER(_i32),
                          C.POINTER(_u16)]),
    "bg_wm_sync": (_int, [_vp, _int, _vp]),
    "bg_wm_classify": (_int, [_vp, _vp, _sz, _sz, _u16, _vp, _vp]),
    "bg_wm_process_host": (_int, [_vp, _vp, _sz, _u16, _vp, _vp]),
    "bg_wm_table_info": (_int, [_vp, C.POINTER(C.c_uint64), C.POINTER(_int)]),
    "bg_wm_jit_wait": (_int, [_vp, _int, _int]),
    "bg_wm_jit_source": (_int, [_vp, _int, _vp, _sz, C.POINTER(_sz)]),
    "bg_wm_jit_check": (_int, [_vp, _vp, _sz, C.POINTER(_sz)]),
    "bg_shutdown": (None, []),
    "bg_stream_attach": (_int, [_vp]),
    "bg_stream_detach": (_int, [_vp]),
    "bg_cksum": (_int, [_int, _vp, _sz, _sz, _int, _int, _vp, _vp, _vp]),
    "bg_cksum_ptrs": (_int, [_int, _vp, _sz, _sz, _int, _int, _vp, _vp, _vp]),
    "bg_host_register": (_int, [_vp, _sz]),
    "bg_host_unregister": (_int, [_vp]),
    "bg_host_dev_addr": (_int, [_vp, _sz, C.POINTER(C.c_uint64)]),
    "bg_cksum_process_host": (_int, [_int, _vp, _sz, _sz, _int, _int, _vp,
                                     _vp, _vp]),
    "bg_module_create": (_int, [C.c_char_p, _vp, _sz, C.POINTER(_vp)]),
    "bg_module_destroy": (None, [_vp]),
    "bg_module_command": (_int, [_vp, C.c_char_p, _vp, _sz, _vp,
                                 C.POINTER(_sz)]),
    "bg_module_process": (_int, [_vp, _vp, _vp, _sz, _vp]),
    "bg_module_process_batches": (_int, [_vp, _vp, _vp, _sz, _vp, _vp, _vp, _vp,
                                         C.POINTER(_sz), C.POINTER(_sz)]),
    "bg_module_connect": (_int, [_vp, _u16, _int]),
    "bg_module_run": (_int, [_vp, _vp, _vp, _sz, _sz, _vp]),
    "bg_module_process_device": (_int, [_vp, _vp, _vp, _sz, _sz, _vp, _vp]),
    "bg_module_set_device": (_int, [_vp, _int]),
    "bg_module_bind_meta": (_int, [_vp, _int, _vp, _vp, _int]),
    "bg_em_bind_meta": (_int, [_vp, _int, _vp, _int]),
    "bg_wm_bind_meta": (_int, [_vp, _int, _vp, _int]),
    "bg_module_desc": (_int, [_vp, C.c_char_p, _sz]),
    "bg_module_attr": (_int, [_vp, _int, C.c_char_p, _sz, C.POINTER(C.c_uint32)]),
    "bg_set_path_flags": (_int, [C.c_uint32]),
    "bg_get_path_flags": (C.c_uint32, []),
    "bg_debug_key": (_int, [C.POINTER(bg_field), _int, _int, _vp, _vp]),
    "bg_em_classify_window": (_int, [_vp, _vp, _sz, _sz, _int, _u16, _vp, _vp]),
    "bg_em_window": (None, [_vp, C.POINTER(_int), C.POINTER(_int)]),
    "bg_wm_classify_window": (_int, [_vp, _vp, _sz, _sz, _int, _u16, _vp, _vp]),
    "bg_wm_window": (None, [_vp, C.POINTER(_int), C.POINTER(_int)]),
    "bg_pipe_create": (_int, [_vp, _int, _sz, _int, _sz, C.POINTER(_vp)]),
    "bg_pipe_destroy": (None, [_vp]),
    "bg_pipe_window": (_int, [_vp, C.POINTER(_int), C.POINTER(_int),
                              C.POINTER(_sz)]),
    "bg_pipe_submit": (_int, [_vp, _vp, _vp, _vp, _vp, _sz]),
    "bg_pipe_submit_meta": (_int, [_vp, _vp, _vp, _vp, _vp, _vp, _sz]),
    "bg_module_process_meta": (_int, [_vp, _vp, _vp, _vp, _sz, _vp]),
    "bg_em_classify_staged": (_int, [_vp, _vp, _sz, _sz, _int, _int, _u16, _vp, _vp]),
    "bg_wm_classify_staged": (_int, [_vp, _vp, _sz, _sz, _int, _int, _u16, _vp, _vp]),
    "bg_em_meta_window": (_int, [_vp, C.POINTER(_int), C.POINTER(_int)]),
    "bg_wm_meta_window": (_int, [_vp, C.POINTER(_int), C.POINTER(_int)]),
    "bg_pipe_flush": (_int, [_vp]),
    "bg_pipe_poll": (C.c_long, [_vp, _int, _vp, _vp, _sz]),
    "bg_pipe_pending": (_sz, [_vp]),
    "bg_pipe_stats": (_int, [_vp, _vp, _int]),
    "bg_pipe_run": (_int, [_vp, _vp, _vp, _vp, _sz, _sz, _vp]),
    "bg_em_ring_create": (_int, [_vp, _int, _int, _int, _int, C.c_uint32, _int,
                                 C.POINTER(_vp)]),
    "bg_wm_ring_create": (_int, [_vp, _int, _int, _int, _int, C.c_uint32, _int,
                                 C.POINTER(_vp)]),
    "bg_ring_destroy": (None, [_vp]),
    "bg_ring_submit": (C.c_int64, [_vp, _int, _vp, _sz, _sz, _u16, _vp]),
    "bg_ring_wait": (_int, [_vp, _int, C.c_int64]),
    "bg_ring_completed": (C.c_int64, [_vp, _int]),
    "bg_ring_run": (_int, [_vp, _int, _vp, _sz, _sz, _sz, _u16, _vp]),
    "bg_ring_run_lanes": (C.c_double, [_vp, _int, _vp, _sz, _sz, _sz, _u16, _vp, _int]),
    "bg_ring_info": (_int, [_vp, C.POINTER(C.c_uint64), C.POINTER(_int)]),
    "bg_ring_desc_in_device": (_int, [_vp]),
    "bg_ring_set_coherence": (_int, [_vp, _int, _int]),
    "bg_hlb_create": (_int, [_int, C.POINTER(bg_field), _int, C.POINTER(_vp)]),
    "bg_hlb_destroy": (None, [_vp]),
    "bg_hlb_set_mode": (_int, [_vp, _int, C.POINTER(bg_field), _int, _int]),
    "bg_hlb_set_gates": (_int, [_vp, _vp, _sz, _sz]),
    "bg_hlb_window": (None, [_vp, C.POINTER(_int), C.POINTER(_int)]),
    "bg_hlb_classify": (_int, [_vp, _vp, _sz, _sz, _int, _vp, _vp]),
    "bg_acl_create": (_int, [C.POINTER(_vp)]),
    "bg_acl_destroy": (None, [_vp]),
    "bg_acl_add": (_int, [_vp, _vp, _sz]),
    "bg_acl_clear": (None, [_vp]),
    "bg_acl_count": (_sz, [_vp]),
    "bg_acl_classify": (_int, [_vp, _vp, _sz, _sz, _u16, _vp, _vp]),
    "bg_acl_tree": (_int, [_vp, _vp, _sz, C.POINTER(_sz), _vp, C.POINTER(C.c_int)]),
    "bg_lpm_create": (_int, [C.c_uint32, C.c_uint32, C.POINTER(_vp)]),
    "bg_lpm_destroy": (None, [_vp]),
    "bg_lpm_add": (_int, [_vp, C.c_uint32, _int, C.c_uint32]),
    "bg_lpm_delete": (_int, [_vp, C.c_uint32, _int]),
    "bg_lpm_clear": (None, [_vp]),
    "bg_lpm_count": (_sz, [_vp]),
    "bg_lpm_classify": (_int, [_vp, _vp, _sz, _sz, _u16, _vp, _vp]),
    "bg_update_ttl": (_int, [_int, _vp, _sz, _sz, _vp, _vp]),
    "bg_ip_encap": (_int, [_int, _vp, _sz, _sz, _int, _vp, _vp, _vp, _vp, _vp]),
    "bg_rewrite_create": (_int, [C.POINTER(_vp)]),
    "bg_rewrite_destroy": (None, [_vp]),
    "bg_rewrite_add": (_int, [_vp, _vp, _vp, _int]),
    "bg_rewrite_clear": (None, [_vp]),
    "bg_rewrite_count": (_sz, [_vp]),
    "bg_rewrite_add_pb": (_int, [_vp, _vp, _sz]),
    "bg_rewrite_process": (_int, [_vp, _int, _vp, _sz, _sz, C.c_uint32, _vp, _vp, _vp]),
    "bg_rewrite_process_host": (_int, [_vp, _int, _vp, _sz, _sz, C.c_uint32, _vp,
                                       _vp, _vp]),
    "bg_dnat_create": (_int, [_vp, _int, _vp, _vp, _vp, _vp, C.c_uint64,
                              C.POINTER(_vp)]),
    "bg_dnat_destroy": (None, [_vp]),
    "bg_dnat_count": (_sz, [_vp]),
    "bg_dnat_process": (_int, [_vp, _vp, _sz, _sz, _int, C.c_uint64, _vp, _vp]),
    "bg_snat_create": (_int, [C.POINTER(_vp)]),
    "bg_snat_destroy": (None, [_vp]),
    "bg_snat_add": (_int, [_vp, C.c_uint32, C.c_uint32, C.c_uint32]),
    "bg_snat_count": (_sz, [_vp]),
    "bg_snat_classify": (_int, [_vp, _vp, _sz, _sz, _int, _vp, _vp]),
}

_lib = None


def lib():
    """Load libbessgpu.so (raises if it has not been built)."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise ImportError(
                "bess_amd: %s missing -- build it (python -c 'import "
                "__graft_entry__ as g; g.build()')" % LIB_PATH)
        # One HIP runtime per process: PyTorch-ROCm ships its own
        # libamdhip64; when it is present it is loaded first so that
        # libbessgpu.so binds to the same runtime (loaded the other way
        # round, the library's runtime reports no device once torch holds
        # the GPU -- measured on the MI355X box)
        try:
            import torch  # noqa: F401
        except ImportError:
            pass
        L = C.CDLL(LIB_PATH)
        for name, (res, args) in _SIGS.items():
            fn = getattr(L, name, None)
            if fn is None:
                continue
            fn.restype = res
            fn.argtypes = args
        _lib = L
        # the run-time compiler thread must be idle before the C-level exit
        # handlers run (bg_shutdown, include/bessgpu.h); Python's atexit
        # hooks run first
        if getattr(L, "bg_shutdown", None) is not None:  # (older builds: none)
            atexit.register(L.bg_shutdown)
    return _lib


class kernel_paths:
    """Context manager: run the enclosed calls with bg_set_path_flags(flags)
    (which of several result-identical kernels serve them), restoring the
    previous flags afterwards."""

    def __init__(self, flags):
        self.flags = flags

    def __enter__(self):
        self.old = lib().bg_get_path_flags()
        check(lib().bg_set_path_flags(self.flags))
        return self

    def __exit__(self, *exc):
        lib().bg_set_path_flags(self.old)
        return False


def check(rc):
    if rc < 0:
        msg = lib().bg_last_error()
        raise BessGpuError(-rc, msg.decode() if msg else "")
    return rc


def declared_symbols():
    """Every function include/bessgpu.h declares (parsed from the header)."""
    import re
    hdr = os.path.join(os.path.dirname(HERE), "include", "bessgpu.h")
    txt = open(hdr).read()
    txt = re.sub(r"/\*.*?\*/", "", txt, flags=re.S)
    return sorted(set(re.findall(r"\b(bg_\w+)\s*\(", txt)))
