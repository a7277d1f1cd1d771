"""pybess-style module handles over libbessgpu's module surface.

    em = ExactMatch(fields=[{'offset': 26, 'num_bytes': 4}, ...])
    em.add(fields=[{'value_bin': b'...'}, ...], gate=1)
    em.set_default_gate(gate=3)
    gates = em.process(frames, stride, n)

Create and command calls carry serialized bess.pb messages through the
bg_module_create / bg_module_command C ABI exactly as pybess carries them
to bessd over gRPC (pybess/bess.py:458-500: `<mclass>Arg` for create, the
command's argument type from the module's cmds table); failures raise
ModuleError(errno, message) like pybess's BESS.Error.
"""
import ctypes as C

import numpy as np

from . import _lib, pb
from ._lib import BG_GATE_NONE, lib, make_ctx

# command -> (argument message, response message or None); module cmds
# tables: exact_match.cc:45-60, wildcard_match.cc:58-73
_EM_CMDS = {
    "get_initial_arg": ("EmptyArg", "ExactMatchArg"),
    "get_runtime_config": ("EmptyArg", "ExactMatchConfig"),
    "set_runtime_config": ("ExactMatchConfig", None),
    "add": ("ExactMatchCommandAddArg", None),
    "delete": ("ExactMatchCommandDeleteArg", None),
    "clear": ("EmptyArg", None),
    "set_default_gate": ("ExactMatchCommandSetDefaultGateArg", None),
}
_WM_CMDS = {
    "get_initial_arg": ("EmptyArg", "WildcardMatchArg"),
    "get_runtime_config": ("EmptyArg", "WildcardMatchConfig"),
    "set_runtime_config": ("WildcardMatchConfig", None),
    "add": ("WildcardMatchCommandAddArg", None),
    "delete": ("WildcardMatchCommandDeleteArg", None),
    "clear": ("EmptyArg", None),
    "set_default_gate": ("WildcardMatchCommandSetDefaultGateArg", None),
}


class ModuleError(RuntimeError):
    def __init__(self, code, msg):
        super().__init__("[errno %d] %s" % (code, msg))
        self.code = code
        self.errmsg = msg


def _check(rc):
    if rc < 0:
        m = lib().bg_last_error()
        raise ModuleError(-rc, m.decode() if m else "")
    return rc


class Module:
    mclass = None
    cmds = {}

    def __init__(self, **kwargs):
        arg = pb.dict_to_protobuf(pb.message(self.mclass + "Arg"), kwargs)
        buf = arg.SerializeToString()
        h = C.c_void_p()
        _check(lib().bg_module_create(self.mclass.encode(), buf, len(buf),
                                      C.byref(h)))
        self.h = h

    def __del__(self):
        if getattr(self, "h", None) is not None and _lib._lib is not None:
            lib().bg_module_destroy(self.h)
            self.h = None

    def command(self, cmd, arg_type=None, **kwargs):
        """bg_module_command with a dict argument; returns the response
        message (or None)."""
        a_type, r_type = self.cmds.get(cmd, (arg_type or "EmptyArg", None))
        arg = pb.dict_to_protobuf(pb.message(a_type), kwargs).SerializeToString()
        cap = C.c_size_t(1 << 16)
        out = C.create_string_buffer(cap.value)
        rc = lib().bg_module_command(self.h, cmd.encode(), arg, len(arg), out,
                                     C.byref(cap))
        if rc < 0 and cap.value > len(out):
            out = C.create_string_buffer(cap.value)
            rc = lib().bg_module_command(self.h, cmd.encode(), arg, len(arg),
                                         out, C.byref(cap))
        _check(rc)
        if r_type is None:
            return None
        return pb.message(r_type).FromString(out.raw[:cap.value])

    def desc(self):
        buf = C.create_string_buffer(256)
        lib().bg_module_desc(self.h, buf, 256)
        return buf.value.decode()

    def set_device(self, device):
        lib().bg_module_set_device(self.h, device)

    def bind_meta(self, meta_off, attr_offsets):
        """attr_name fields (ExactMatch, WildcardMatch): each slot carries
        the packet's metadata area at byte meta_off; attr_offsets maps an
        attribute name to the metadata offset the pipeline assigned it
        (Module::attr_offset, core/module.h)."""
        names = list(attr_offsets)
        arr = (C.c_char_p * max(len(names), 1))(*[n.encode() for n in names])
        offs = (C.c_int32 * max(len(names), 1))(*[int(attr_offsets[n]) for n in names])
        _check(lib().bg_module_bind_meta(self.h, meta_off, arr, offs, len(names)))

    def process_meta(self, heads, metas, igate=0, now=None, device=-1):
        """ProcessBatch over host packets given by head_data() and metadata
        area addresses (numpy uintp arrays; bg_module_process_meta)"""
        heads = np.ascontiguousarray(heads, dtype=np.uintp)
        metas = np.ascontiguousarray(metas, dtype=np.uintp)
        n = len(heads)
        og = np.full(n, BG_GATE_NONE, np.uint16)
        _check(lib().bg_module_process_meta(self.h, make_ctx(igate, now, device),
                                            heads.ctypes.data, metas.ctypes.data, n,
                                            og.ctypes.data))
        return og

    def process(self, frames, stride, n, igate=0, now=None, device=-1):
        """ProcessBatch over host frames (numpy uint8 slab, frame i at
        i*stride, each with >= 2048 accessible bytes for the checksum
        modules) with the call's context (ctx->current_igate, current_ns,
        core/module.h:59-75; now None = the library's clock). Returns
        per-packet EmitPacket gates (BG_GATE_NONE: not emitted). Checksum
        modules rewrite frames in place."""
        base = frames.ctypes.data
        heads = (C.c_void_p * n)(*[base + i * stride for i in range(n)])
        og = np.full(n, BG_GATE_NONE, np.uint16)
        _check(lib().bg_module_process(self.h, make_ctx(igate, now, device), heads,
                                       n, og.ctypes.data))
        return og

    def process_batches(self, frames, stride, n, igate=0, now=None):
        """process() plus the batches the Task would run next
        (core/module.h:543-618): -> (ogates, [(gate, [packet index, ...])],
        [dropped packet index, ...])"""
        base = frames.ctypes.data
        heads = (C.c_void_p * n)(*[base + i * stride for i in range(n)])
        og = np.full(n, BG_GATE_NONE, np.uint16)
        bg_ = np.zeros(max(n, 1), np.uint16)
        bl = np.zeros(max(n, 1), np.uint32)
        idx = np.zeros(max(n, 1), np.uint32)
        nb, nd = C.c_size_t(), C.c_size_t()
        _check(lib().bg_module_process_batches(
            self.h, make_ctx(igate, now), heads, n, og.ctypes.data, bg_.ctypes.data, bl.ctypes.data,
            idx.ctypes.data, C.byref(nb), C.byref(nd)))
        batches, k = [], 0
        for b in range(nb.value):
            batches.append((int(bg_[b]), [int(x) for x in idx[k:k + bl[b]]]))
            k += int(bl[b])
        return og, batches, [int(x) for x in idx[k:k + nd.value]]

    def run(self, heads, burst=32, igate=0, now=None, device=-1):
        """a worker's synchronous loop (bg_module_run) over head addresses
        (numpy uintp) in bursts; -> gates"""
        heads = np.ascontiguousarray(heads, dtype=np.uintp)
        og = np.full(len(heads), BG_GATE_NONE, np.uint16)
        _check(lib().bg_module_run(self.h, make_ctx(igate, now, device),
                                   heads.ctypes.data, len(heads), burst,
                                   og.ctypes.data))
        return og

    def connect(self, ogate, connected=True):
        """ogate connected to a next module or not (ConnectModules); until
        the first call every gate counts as connected"""
        _check(lib().bg_module_connect(self.h, ogate, 1 if connected else 0))

    def process_device(self, d_frames, stride, n, d_ogates, stream=None, igate=0,
                       now=None):
        """Device-resident ProcessBatch over a torch uint8 slab (on the
        module's device)."""
        from .flowtable import _stream_ptr
        _check(lib().bg_module_process_device(
            self.h, make_ctx(igate, now), C.c_void_p(d_frames.data_ptr()), stride, n,
            C.c_void_p(d_ogates.data_ptr()), _stream_ptr(stream)))


class _RuleModule(Module):
    def get_initial_arg(self):
        return self.command("get_initial_arg")

    def get_runtime_config(self):
        return self.command("get_runtime_config")

    def set_runtime_config(self, **kw):
        return self.command("set_runtime_config", **kw)

    def add(self, **kw):
        return self.command("add", **kw)

    def delete(self, **kw):
        return self.command("delete", **kw)

    def clear(self):
        return self.command("clear")

    def set_default_gate(self, **kw):
        return self.command("set_default_gate", **kw)


class ExactMatch(_RuleModule):
    """core/modules/exact_match.cc on the GPU."""
    mclass = "ExactMatch"
    cmds = _EM_CMDS


class WildcardMatch(_RuleModule):
    """core/modules/wildcard_match.cc on the GPU."""
    mclass = "WildcardMatch"
    cmds = _WM_CMDS


class IPChecksum(Module):
    """core/modules/ip_checksum.cc on the GPU."""
    mclass = "IPChecksum"


class L4Checksum(Module):
    """core/modules/l4_checksum.cc on the GPU."""
    mclass = "L4Checksum"


class HashLB(Module):
    """core/modules/hash_lb.cc on the GPU."""
    mclass = "HashLB"
    cmds = {"set_mode": ("HashLBCommandSetModeArg", None),
            "set_gates": ("HashLBCommandSetGatesArg", None)}

    def set_mode(self, **kw):
        return self.command("set_mode", **kw)

    def set_gates(self, **kw):
        return self.command("set_gates", **kw)


class ACL(Module):
    """core/modules/acl.cc on the GPU."""
    mclass = "ACL"
    cmds = {"add": ("ACLArg", None), "clear": ("EmptyArg", None)}

    def add(self, **kw):
        return self.command("add", **kw)

    def clear(self):
        return self.command("clear")


class IPLookup(Module):
    """core/modules/ip_lookup.cc on the GPU."""
    mclass = "IPLookup"
    cmds = {"add": ("IPLookupCommandAddArg", None),
            "delete": ("IPLookupCommandDeleteArg", None),
            "clear": ("EmptyArg", None)}

    def add(self, **kw):
        return self.command("add", **kw)

    def delete(self, **kw):
        return self.command("delete", **kw)

    def clear(self):
        return self.command("clear")


class UpdateTTL(Module):
    """core/modules/update_ttl.cc on the GPU."""
    mclass = "UpdateTTL"


class StaticNAT(Module):
    """core/modules/static_nat.cc on the GPU: input gate 0 translates the
    source (emits on 1), input gate 1 the destination (emits on 0)."""
    mclass = "StaticNAT"
    cmds = {"get_initial_arg": ("EmptyArg", "StaticNATArg"),
            "get_runtime_config": ("EmptyArg", None),
            "set_runtime_config": ("EmptyArg", None)}

    def get_initial_arg(self):
        return self.command("get_initial_arg")


def _nat_arrays(ext_addrs):
    """NATArg.ext_addrs (module_msg.proto) -> flat C arrays"""
    addrs, nr, beg, end, sus = [], [], [], [], []
    for a in ext_addrs:
        addrs.append(str(a.get("ext_addr", "")).encode())
        rl = a.get("port_ranges", [])
        nr.append(len(rl))
        for r in rl:
            beg.append(int(r.get("begin", 0)))
            end.append(int(r.get("end", 0)))
            sus.append(1 if r.get("suspended", False) else 0)
    k = max(len(beg), 1)
    return ((C.c_char_p * max(len(addrs), 1))(*addrs), len(addrs),
            (C.c_int32 * max(len(nr), 1))(*nr), (C.c_int64 * k)(*beg),
            (C.c_int64 * k)(*end), (C.c_uint8 * k)(*sus))


class NAT:
    """core/modules/nat.cc on the GPU (bg_dnat_*): NAT(ext_addrs=[{'ext_addr':
    '1.2.3.4', 'port_ranges': [{'begin': b, 'end': e, 'suspended': s}]}],
    seed=...) -- the reference seeds its port search from rdtsc."""

    def __init__(self, ext_addrs=(), seed=0x5EED):
        a, n, nr, b, e, s = _nat_arrays(ext_addrs)
        h = C.c_void_p()
        _check(lib().bg_dnat_create(a, n, nr, b, e, s, seed, C.byref(h)))
        self.h = h

    def __del__(self):
        if getattr(self, "h", None) is not None and _lib._lib is not None:
            lib().bg_dnat_destroy(self.h)
            self.h = None

    def desc(self):
        return "%d entries" % lib().bg_dnat_count(self.h)

    def process_device(self, d_frames, stride, n, d_ogates, now, igate=0,
                       stream=None):
        from .flowtable import _stream_ptr
        _check(lib().bg_dnat_process(self.h, C.c_void_p(d_frames.data_ptr()), stride,
                                     n, 0 if igate == 0 else 1, now,
                                     C.c_void_p(d_ogates.data_ptr()),
                                     _stream_ptr(stream)))


# IPEncap attribute order (ip_encap.cc:36-40)
IP_ENCAP_ATTRS = ("ip_src", "ip_dst", "ip_proto", "ip_nexthop", "ether_type")


def ip_encap(d_slots, stride, n, meta_off, attr_offsets, d_head, d_len, d_out,
             device=0, stream=None):
    """core/modules/ip_encap.cc on the GPU (bg_ip_encap): torch tensors
    d_slots (uint8 slab), d_head (int16: data_off), d_len (int32: pkt_len),
    d_out (int16 gates); attr_offsets maps IP_ENCAP_ATTRS names to the
    attribute offsets in the metadata area (missing: invalid)."""
    from .flowtable import _stream_ptr
    offs = (C.c_int32 * 5)(*[int(attr_offsets.get(k, -1)) for k in IP_ENCAP_ATTRS])
    _check(lib().bg_ip_encap(device, C.c_void_p(d_slots.data_ptr()), stride, n,
                             meta_off, offs, C.c_void_p(d_head.data_ptr()),
                             C.c_void_p(d_len.data_ptr()),
                             C.c_void_p(d_out.data_ptr()), _stream_ptr(stream)))


class Rewrite:
    """core/modules/rewrite.{h,cc} on the GPU (bg_rewrite_*): Init(arg) =
    add(arg.templates); the add / clear commands; ProcessBatch over a device
    slab of packet slots or over host packet buffers."""
    mclass = "Rewrite"
    cmds = {"add": ("RewriteArg", "EmptyArg"), "clear": ("EmptyArg", "EmptyArg")}
    SNBUF_HEADROOM = 128

    def __init__(self, templates=()):
        h = C.c_void_p()
        _check(lib().bg_rewrite_create(C.byref(h)))
        self.h = h
        self.add(templates=templates)

    def __del__(self):
        if getattr(self, "h", None) is not None and _lib._lib is not None:
            lib().bg_rewrite_destroy(self.h)
            self.h = None

    def add(self, templates=()):
        """RewriteArg.templates: bytes"""
        ts = [bytes(t) for t in templates]
        bufs = [C.create_string_buffer(t, max(len(t), 1)) for t in ts]
        ptrs = (C.c_void_p * max(len(ts), 1))(*[C.addressof(b) for b in bufs])
        lens = (C.c_uint32 * max(len(ts), 1))(*[len(t) for t in ts])
        _check(lib().bg_rewrite_add(self.h, ptrs, lens, len(ts)))

    def clear(self):
        lib().bg_rewrite_clear(self.h)

    def __len__(self):
        return lib().bg_rewrite_count(self.h)

    def process_device(self, d_slots, stride, n, d_head, d_len,
                       headroom=SNBUF_HEADROOM, device=0, stream=None):
        """torch tensors: d_slots (uint8 slab), d_head (int16: data_off),
        d_len (int32: pkt_len)"""
        from .flowtable import _stream_ptr
        _check(lib().bg_rewrite_process(self.h, device, C.c_void_p(d_slots.data_ptr()),
                                        stride, n, headroom,
                                        C.c_void_p(d_head.data_ptr()),
                                        C.c_void_p(d_len.data_ptr()), _stream_ptr(stream)))

    def process_host(self, slots, slot_bytes, head, length, headroom=SNBUF_HEADROOM,
                     device=0):
        """slots: array of buffer addresses (uintp); head uint16 / length
        uint32 numpy arrays, written"""
        n = len(slots)
        ptrs = np.ascontiguousarray(slots, dtype=np.uintp)
        _check(lib().bg_rewrite_process_host(self.h, device, ptrs.ctypes.data, slot_bytes,
                                             n, headroom, head.ctypes.data,
                                             length.ctypes.data, None))


class Pipe:
    """Asynchronous host ingress/egress for a module (bg_pipe_*): packets
    are submitted in BESS-sized batches (<= 32 per ProcessBatch), gathered
    into pinned slots of `batch` packets, launched H2D -> device -> D2H on
    `depth` streams, and returned by poll() in submission order with their
    EmitPacket gate (core/modules/queue.cc:173/190 split)."""

    def __init__(self, module, device=0, batch=4096, depth=4, span=0):
        h = C.c_void_p()
        _check(lib().bg_pipe_create(module.h, device, batch, depth, span,
                                    C.byref(h)))
        self.h = h
        self.module = module  # keep the module alive while the pipe is

    def close(self):
        if getattr(self, "h", None) is not None and _lib._lib is not None:
            lib().bg_pipe_destroy(self.h)
            self.h = None

    __del__ = close

    def window(self):
        lo, hi, st = C.c_int(), C.c_int(), C.c_size_t()
        lib().bg_pipe_window(self.h, C.byref(lo), C.byref(hi), C.byref(st))
        return lo.value, hi.value, st.value

    def submit(self, heads, lens=None, cookies=None, igate=0, now=None, metas=None):
        """heads: numpy uintp array of head_data() addresses; igate / now:
        the ProcessBatch's context; metas: the packets' metadata areas
        (modules with attr_name fields)."""
        heads = np.ascontiguousarray(heads, dtype=np.uintp)
        n = len(heads)
        if metas is not None:
            metas = np.ascontiguousarray(metas, dtype=np.uintp)
        lp = None
        if lens is not None:
            lens = np.ascontiguousarray(lens, dtype=np.uint16)
            lp = lens.ctypes.data
        cp = None
        if cookies is not None:
            cookies = np.ascontiguousarray(cookies, dtype=np.uintp)
            cp = cookies.ctypes.data
        if metas is None:
            _check(lib().bg_pipe_submit(self.h, make_ctx(igate, now), heads.ctypes.data,
                                        lp, cp, n))
        else:
            _check(lib().bg_pipe_submit_meta(self.h, make_ctx(igate, now), heads.ctypes.data,
                                             metas.ctypes.data, lp, cp, n))

    def flush(self):
        _check(lib().bg_pipe_flush(self.h))

    def poll(self, wait=False, cap=1 << 16):
        """-> (cookies uintp array, gates uint16 array)"""
        ck = np.empty(cap, np.uintp)
        g = np.empty(cap, np.uint16)
        k = _check(lib().bg_pipe_poll(self.h, 1 if wait else 0, ck.ctypes.data,
                                      g.ctypes.data, cap))
        return ck[:k], g[:k]

    def pending(self):
        return lib().bg_pipe_pending(self.h)

    def run(self, heads, lens=None, burst=32, igate=0, now=None):
        """native worker loop over all packets (bg_pipe_run); -> gates"""
        heads = np.ascontiguousarray(heads, dtype=np.uintp)
        n = len(heads)
        og = np.full(n, BG_GATE_NONE, np.uint16)
        lp = None
        if lens is not None:
            lens = np.ascontiguousarray(lens, dtype=np.uint16)
            lp = lens.ctypes.data
        _check(lib().bg_pipe_run(self.h, make_ctx(igate, now), heads.ctypes.data,
                                 lp, n, burst,
                                 og.ctypes.data))
        return og

    def drain(self):
        """flush and wait for everything submitted"""
        self.flush()
        cs, gs = [], []
        while self.pending():
            c, g = self.poll(wait=True)
            cs.append(c)
            gs.append(g)
        if not cs:
            return np.empty(0, np.uintp), np.empty(0, np.uint16)
        return np.concatenate(cs), np.concatenate(gs)
