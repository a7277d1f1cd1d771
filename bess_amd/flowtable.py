"""Python face of the device flow tables (bg_em / bg_wm / bg_cksum).

Thin wrappers over include/bessgpu.h. Device buffers are torch tensors on a
HIP device (torch is plumbing: memory, streams, RCCL); every byte of
classification work runs in libbessgpu.so's gfx950 kernels.
"""
import ctypes as C

import numpy as np

from . import _lib
from ._lib import BessGpuError, bg_field, check, lib

__all__ = ["Comm", "EmTable", "Ring", "WmTable", "cksum", "cksum_host", "resolve_em_fields",
           "resolve_wm_fields", "BessGpuError"]


def _stream_ptr(stream):
    if stream is None:
        import torch
        return C.c_void_p(torch.cuda.current_stream().cuda_stream)
    if isinstance(stream, int):
        return C.c_void_p(stream)
    return C.c_void_p(stream.cuda_stream)


def _dev_ptr(t):
    return C.c_void_p(t.data_ptr())


def resolve_em_fields(specs):
    """[(offset, size, mask)] -> bg_field array with key positions (the
    resolved ExactMatchField of exact_match_table.h:126-140)."""
    arr = (bg_field * max(len(specs), 1))()
    pos = 0
    for i, (off, size, mask) in enumerate(specs):
        arr[i].offset, arr[i].size, arr[i].pos = off, size, pos
        arr[i].attr_id, arr[i].mask = -1, mask
        pos += size
    return arr, len(specs)


def resolve_wm_fields(specs):
    """[(offset, size)] -> bg_field array (WmField, wildcard_match.h:62-72)."""
    return resolve_em_fields([(o, s, 0) for o, s in specs])


class EmTable:
    """bg_em: ExactMatchTable<gate_idx_t> with a device image."""

    def __init__(self, fields):
        """fields: [(offset, size, mask)] with mask = ExactMatchField::mask
        (key byte order, low `size` bytes)."""
        arr, n = resolve_em_fields(fields)
        h = C.c_void_p()
        check(lib().bg_em_create(arr, n, C.byref(h)))
        self.h = h
        self.key_size = lib().bg_em_key_size(h)

    def __del__(self):
        if getattr(self, "h", None) is not None and _lib._lib is not None:
            lib().bg_em_destroy(self.h)
            self.h = None

    def add(self, key, gate):
        check(lib().bg_em_add(self.h, bytes(key).ljust(64, b"\0"), gate))

    def add_many(self, keys, gates, part=-1, nparts=1):
        """keys: (n, key_size) uint8 array; gates: (n,) ints. part >= 0:
        keep only the rules of partition `part` of an nparts-way sharded
        table (a multi-GPU rank's share)."""
        keys = np.ascontiguousarray(keys, dtype=np.uint8)
        if keys.shape[1] < self.key_size:
            keys = np.ascontiguousarray(np.pad(
                keys, ((0, 0), (0, self.key_size - keys.shape[1]))))
        g = np.ascontiguousarray(gates, dtype=np.uint16)
        check(lib().bg_em_add_many(self.h, keys.ctypes.data, len(keys),
                                   keys.shape[1], g.ctypes.data, part, nparts))

    def part_count(self, part, nparts):
        c = C.c_uint64()
        check(lib().bg_em_part_count(self.h, part, nparts, C.byref(c)))
        return c.value

    def plan_count(self, nparts, max_part_entries):
        pb = C.c_uint64()
        check(lib().bg_em_plan_count(self.h, nparts, max_part_entries,
                                     C.byref(pb)))
        return pb.value

    def delete(self, key):
        check(lib().bg_em_delete(self.h, bytes(key).ljust(64, b"\0")))

    def clear(self):
        lib().bg_em_clear(self.h)

    def __len__(self):
        return lib().bg_em_count(self.h)

    def sync(self, device=0, stream=None):
        check(lib().bg_em_sync(self.h, device, _stream_ptr(stream)))

    def classify(self, frames, stride, n, default_gate, gates, stream=None):
        """frames: device uint8 tensor (slab); gates: device int16/uint16."""
        check(lib().bg_em_classify(self.h, _dev_ptr(frames), stride, n,
                                   default_gate, _dev_ptr(gates),
                                   _stream_ptr(stream)))

    def process_host(self, frames_np, stride, n, default_gate, stream=None):
        """Host frames (numpy slab) through the staged host path."""
        base = frames_np.ctypes.data
        heads = (C.c_void_p * n)(*[base + i * stride for i in range(n)])
        out = np.zeros(n, np.uint16)
        check(lib().bg_em_process_host(self.h, heads, n, default_gate,
                                       out.ctypes.data, _stream_ptr(stream)))
        return out

    def plan(self, nparts):
        pb = C.c_uint64()
        check(lib().bg_em_plan(self.h, nparts, C.byref(pb)))
        return pb.value

    def build_part(self, part, nbytes):
        buf = np.zeros(nbytes, np.uint8)
        check(lib().bg_em_build_part(self.h, part, buf.ctypes.data))
        return buf

    def attach(self, device, d_image):
        check(lib().bg_em_attach(self.h, device, _dev_ptr(d_image)))

    def table_info(self):
        b, l = C.c_uint64(), C.c_int()
        check(lib().bg_em_table_info(self.h, C.byref(b), C.byref(l)))
        return b.value, bool(l.value)

    def allgather(self, comm, stream=None):
        """bg_em_allgather: this rank's share of the sharded build over RCCL;
        the assembled image becomes the table's image on comm's device"""
        check(lib().bg_em_allgather(self.h, comm.h, _stream_ptr(stream)))

    def allgather_all(self, comms):
        """bg_em_allgather_all: every rank of an init_all set, one thread"""
        arr = (C.c_void_p * len(comms))(*[c.h.value for c in comms])
        check(lib().bg_em_allgather_all(self.h, arr, len(comms)))


class Comm:
    """bg_comm: one rank of an RCCL communicator over the GPUs that share a
    rule set (the C ABI's own, no torch.distributed)."""

    def __init__(self, h):
        self.h = h

    @staticmethod
    def unique_id():
        buf = (C.c_uint8 * 128)()
        check(lib().bg_comm_unique_id(buf))
        return bytes(buf)

    @classmethod
    def init_rank(cls, uid, nranks, rank, device):
        h = C.c_void_p()
        buf = (C.c_uint8 * 128)(*uid)
        check(lib().bg_comm_init_rank(buf, nranks, rank, device, C.byref(h)))
        return cls(h)

    @classmethod
    def init_all(cls, devices):
        devs = (C.c_int * len(devices))(*devices)
        hs = (C.c_void_p * len(devices))()
        check(lib().bg_comm_init_all(devs, len(devices), hs))
        return [cls(C.c_void_p(h)) for h in hs]

    def info(self):
        r, n, d = C.c_int(), C.c_int(), C.c_int()
        check(lib().bg_comm_info(self.h, C.byref(r), C.byref(n), C.byref(d)))
        return r.value, n.value, d.value

    def last_stats(self):
        """the rank's last EmTable.allgather: {"allreduce_ms", "build_ms",
        "allgather_ms", "bytes"} (bg_comm_last_stats)"""
        ns = (C.c_uint64 * 3)()
        b = C.c_uint64()
        check(lib().bg_comm_last_stats(self.h, ns, C.byref(b)))
        return {"allreduce_ms": ns[0] / 1e6, "build_ms": ns[1] / 1e6,
                "allgather_ms": ns[2] / 1e6, "bytes": b.value}

    @classmethod
    def over_process_group(cls, rank, world, device, dist, group=None):
        """one rank of a communicator for `world` processes: rank 0's unique
        id travels over the caller's existing torch.distributed group (128
        control bytes; the table itself never goes through torch)"""
        uid = [None]
        if rank == 0:
            try:
                uid[0] = cls.unique_id()
            except Exception as e:  # every rank learns it (none waits in init)
                uid[0] = "bg_comm_unique_id failed: %r" % (e,)
        dist.broadcast_object_list(uid, src=0, group=group)
        if not isinstance(uid[0], (bytes, bytearray)):
            raise RuntimeError(str(uid[0]))
        return cls.init_rank(uid[0], world, rank, device)

    def close(self):
        if getattr(self, "h", None) is not None and _lib._lib is not None:
            lib().bg_comm_destroy(self.h)
            self.h = None

    __del__ = close


class Ring:
    """bg_ring: one persistent ExactMatch (or WildcardMatch: bg_wm_ring_create)
    kernel draining batch descriptors
    from `lanes` submission lanes, one per worker thread (the table as of
    creation, in LDS for the kernel's whole run)."""

    def __init__(self, table, device=0, slots=1024, blocks=0, idle_us=200000,
                 lanes=1, win_off=0):
        h = C.c_void_p()
        create = (lib().bg_wm_ring_create if isinstance(table, WmTable)
                  else lib().bg_em_ring_create)
        check(create(table.h, device, lanes, slots, blocks, idle_us, win_off, C.byref(h)))
        self.h = h
        self.table = table
        self.lanes = lanes
        self.device = device

    def close(self):
        if getattr(self, "h", None) is not None and _lib._lib is not None:
            lib().bg_ring_destroy(self.h)
            self.h = None

    __del__ = close

    def submit(self, frames, stride, n, default_gate, gates, offset=0, lane=0):
        """frames / gates: device tensors; batch = packets [offset, offset+n)"""
        t = lib().bg_ring_submit(self.h, lane,
                                 C.c_void_p(frames.data_ptr() + offset * stride),
                                 stride, n, default_gate,
                                 C.c_void_p(gates.data_ptr() + 2 * offset))
        return check(t)

    def wait(self, ticket, lane=0):
        check(lib().bg_ring_wait(self.h, lane, ticket))

    def completed(self, lane=0):
        return check(lib().bg_ring_completed(self.h, lane))

    def run(self, frames, stride, n, burst, default_gate, gates, lane=0, offset=0):
        """packets [offset, offset + n) in batches of `burst` on one lane"""
        check(lib().bg_ring_run(self.h, lane,
                                C.c_void_p(frames.data_ptr() + offset * stride),
                                stride, n, burst, default_gate,
                                C.c_void_p(gates.data_ptr() + 2 * offset)))

    def run_lanes(self, frames, stride, n, burst, default_gate, gates, threads, reps=1):
        """`threads` submitters at once (threads <= lanes; native threads,
        bg_ring_run_lanes), thread i on lane i over packets
        [i*n/threads, (i+1)*n/threads), `reps` passes each; -> wall seconds
        per pass"""
        dt = lib().bg_ring_run_lanes(self.h, threads, C.c_void_p(frames.data_ptr()),
                                     stride, n, burst, default_gate,
                                     C.c_void_p(gates.data_ptr()), reps)
        if dt < 0:
            raise BessGpuError(-int(dt), lib().bg_last_error().decode())
        return dt

    def set_coherence(self, frames, done):
        """bg_ring_set_coherence: frames 0 for device memory written by
        kernels or uncached host memory (1: any memory); done 1 for a
        system-scope release on the done word"""
        check(lib().bg_ring_set_coherence(self.h, int(frames), int(done)))

    def info(self):
        launches, blocks = C.c_uint64(), C.c_int()
        lib().bg_ring_info(self.h, C.byref(launches), C.byref(blocks))
        return launches.value, blocks.value

    def desc_in_device(self):
        """True: descriptors in device memory the host writes (BAR)."""
        return bool(lib().bg_ring_desc_in_device(self.h))


class WmTable:
    """bg_wm: WildcardMatch tuple tables with a device image."""

    def __init__(self, fields):
        """fields: [(offset, size)]"""
        arr, n = resolve_wm_fields(fields)
        h = C.c_void_p()
        check(lib().bg_wm_create(arr, n, C.byref(h)))
        self.h = h
        self.key_size = lib().bg_wm_key_size(h)

    def __del__(self):
        if getattr(self, "h", None) is not None and _lib is not None and _lib._lib is not None:
            lib().bg_wm_destroy(self.h)
            self.h = None

    def add(self, key, mask, priority, gate):
        check(lib().bg_wm_add(self.h, bytes(key).ljust(64, b"\0"),
                              bytes(mask).ljust(64, b"\0"), priority, gate))

    def delete(self, key, mask):
        check(lib().bg_wm_delete(self.h, bytes(key).ljust(64, b"\0"),
                                 bytes(mask).ljust(64, b"\0")))

    def clear(self):
        lib().bg_wm_clear(self.h)

    def num_tuples(self):
        return lib().bg_wm_num_tuples(self.h)

    def sync(self, device=0, stream=None):
        check(lib().bg_wm_sync(self.h, device, _stream_ptr(stream)))

    def classify(self, frames, stride, n, default_gate, gates, stream=None):
        check(lib().bg_wm_classify(self.h, _dev_ptr(frames), stride, n,
                                   default_gate, _dev_ptr(gates),
                                   _stream_ptr(stream)))

    def process_host(self, frames_np, stride, n, default_gate, stream=None):
        base = frames_np.ctypes.data
        heads = (C.c_void_p * n)(*[base + i * stride for i in range(n)])
        out = np.zeros(n, np.uint16)
        check(lib().bg_wm_process_host(self.h, heads, n, default_gate,
                                       out.ctypes.data, _stream_ptr(stream)))
        return out

    def table_info(self):
        b, l = C.c_uint64(), C.c_int()
        check(lib().bg_wm_table_info(self.h, C.byref(b), C.byref(l)))
        # 0 L2/MALL, 1 table in LDS, 2 key filter in LDS, 3 tag words in LDS
        return b.value, l.value & 0xFF

    def jit_wait(self, device=0, timeout_ms=120000):
        """Block until the run-time compiled kernel of the current rules is
        ready on `device` (bg_wm_jit_wait)."""
        check(lib().bg_wm_jit_wait(self.h, device, timeout_ms))

    def jit_source(self, device=0):
        need = C.c_size_t()
        check(lib().bg_wm_jit_source(self.h, device, None, 0, C.byref(need)))
        buf = C.create_string_buffer(need.value)
        check(lib().bg_wm_jit_source(self.h, device, buf, need.value, C.byref(need)))
        return buf.value.decode()

    def jit_check(self):
        """Compile the specialised kernel of the current rules on this thread
        (no device): (rc, code bytes, compiler log)."""
        log = C.create_string_buffer(1 << 16)
        cb = C.c_size_t()
        rc = lib().bg_wm_jit_check(self.h, log, len(log), C.byref(cb))
        return rc, cb.value, log.value.decode(errors="replace")

    def direct_tuples(self):
        """tuples of the device image read by index (one- or two-byte masks)"""
        b, l = C.c_uint64(), C.c_int()
        check(lib().bg_wm_table_info(self.h, C.byref(b), C.byref(l)))
        return l.value >> 8


def cksum(frames, stride, n, mode, verify, ip_gates=None, l4_gates=None,
          device=0, stream=None):
    """IPChecksum (mode 1) / L4Checksum (mode 2) / both (3) on a device slab,
    in place."""
    check(lib().bg_cksum(device, _dev_ptr(frames), stride, n, mode,
                         1 if verify else 0,
                         _dev_ptr(ip_gates) if ip_gates is not None else None,
                         _dev_ptr(l4_gates) if l4_gates is not None else None,
                         _stream_ptr(stream)))


def cksum_ptrs(d_ptrs, span, n, mode, verify, ip_gates=None, l4_gates=None,
               device=0, stream=None):
    """IPChecksum / L4Checksum on frames by pointer (d_ptrs: a device
    uint64 tensor of device addresses, e.g. of host-registered memory), in
    place."""
    check(lib().bg_cksum_ptrs(device, _dev_ptr(d_ptrs), span, n, mode,
                              1 if verify else 0,
                              _dev_ptr(ip_gates) if ip_gates is not None else None,
                              _dev_ptr(l4_gates) if l4_gates is not None else None,
                              _stream_ptr(stream)))


class HostRegion:
    """Host memory registered for in-place device access (bg_host_register);
    `addr(p)` is the device address of host address p."""

    def __init__(self, arr):
        self.arr = arr  # kept alive while registered
        self.base = arr.ctypes.data
        check(lib().bg_host_register(C.c_void_p(self.base), arr.nbytes))

    def addr(self, p, length=1):
        d = C.c_uint64()
        check(lib().bg_host_dev_addr(C.c_void_p(int(p)), length, C.byref(d)))
        return d.value

    def close(self):
        if self.arr is not None:
            check(lib().bg_host_unregister(C.c_void_p(self.base)))
            self.arr = None


def cksum_host(frames_np, stride, n, mode, verify, span=None, device=0,
               stream=None):
    """Host slab through the staged host path (in place); returns gates."""
    span = stride if span is None else span
    base = frames_np.ctypes.data
    heads = (C.c_void_p * n)(*[base + i * stride for i in range(n)])
    ipg = np.zeros(n, np.uint16)
    l4g = np.zeros(n, np.uint16)
    check(lib().bg_cksum_process_host(device, heads, n, span, mode,
                                      1 if verify else 0, ipg.ctypes.data,
                                      l4g.ctypes.data, _stream_ptr(stream)))
    return ipg, l4g
