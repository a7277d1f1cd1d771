"""TEST INFRASTRUCTURE ONLY: control-plane restatements of the SURVEY §8f
modules (HashLB, ACL, IPLookup, UpdateTTL, StaticNAT, IPEncap, NAT) around oracle_more.c. Only
tests/, smoke() and bench.py's cpu_baseline leg import this. Each method
cites the reference file:line it follows; errors raise OracleError(errno,
message) with the reference's text."""
import ctypes as C
import errno as E

import numpy as np

from .oracle import OracleError, lib, _ptr

_sz, _vp = C.c_size_t, C.c_void_p
class or_acl_rule(C.Structure):
    _fields_ = [("src_addr", C.c_uint32), ("src_mask", C.c_uint32),
                ("dst_addr", C.c_uint32), ("dst_mask", C.c_uint32),
                ("src_port", C.c_uint16), ("dst_port", C.c_uint16),
                ("drop", C.c_uint8), ("pad", C.c_uint8 * 3)]


_SIGS = {
    "or_ipv4_address": (C.c_int, [C.c_char_p, C.POINTER(C.c_uint32)]),
    "or_ipv4_prefix": (C.c_int, [C.c_char_p, C.POINTER(C.c_uint32),
                                 C.POINTER(C.c_uint32)]),
    "or_acl_process": (None, [_vp, _sz, _vp, _sz, _sz, C.c_uint16, _vp]),
    "or_acl_bench": (C.c_double, [_vp, _sz, _vp, _sz, _sz, C.c_uint16, _vp,
                                  C.c_int, C.c_int]),
    "or_em_make_key": (None, [_vp, _vp, _vp]),
    "or_update_ttl_process": (None, [_vp, _sz, _sz, _vp]),
    "or_static_nat_process": (None, [_vp, _vp, _vp, _sz, _vp, _sz, _sz, C.c_int,
                                     _vp]),
    "or_ip_encap_process": (None, [_vp, _sz, _sz, C.c_int, _vp, _vp, _vp, _vp]),
    "or_rewrite_new": (_vp, []),
    "or_rewrite_free": (None, [_vp]),
    "or_rewrite_add": (C.c_int, [_vp, _vp, _vp, C.c_int, C.c_char_p, _sz]),
    "or_rewrite_clear": (None, [_vp]),
    "or_rewrite_process": (None, [_vp, _vp, _sz, _sz, C.c_uint32, _vp, _vp]),
    "or_nat_new": (_vp, [C.c_uint64]),
    "or_nat_free": (None, [_vp]),
    "or_nat_count": (_sz, [_vp]),
    "or_nat_init": (None, [_vp, _vp, C.c_uint32, _vp, _vp, _vp, _vp]),
    "or_nat_process": (None, [_vp, _vp, _sz, _sz, C.c_int, C.c_uint64, _vp]),
    "or_lpm_process": (None, [_vp, _vp, _vp, _sz, _vp, _sz, _sz, C.c_uint16,
                              _vp]),
    "or_hash_range": (C.c_uint16, [C.c_uint32, C.c_uint16]),
    "or_dir24_build": (_vp, [_vp, _vp, _vp, _sz]),
    "or_dir24_free": (None, [_vp]),
    "or_dir24_process": (None, [_vp, _vp, _sz, _sz, C.c_uint16, _vp]),
    "or_dir24_bench": (C.c_double, [_vp, _vp, _sz, _sz, C.c_uint16, _vp,
                                    C.c_int, C.c_int]),
    "or_update_ttl_bench": (C.c_double, [_vp, _sz, _sz, _vp, C.c_int, C.c_int]),
    "or_static_nat_bench": (C.c_double, [_vp, _vp, _vp, _sz, _vp, _sz, _sz, _vp,
                                         C.c_int, C.c_int]),
    "or_hashlb_process": (None, [C.c_int, _vp, _sz, _vp, _sz, _vp, _sz, _sz,
                                 _vp]),
    "or_hashlb_bench": (C.c_double, [C.c_int, _vp, _sz, _vp, _sz, _vp, _sz,
                                     _sz, _vp, C.c_int, C.c_int]),
}
_done = False


def mlib():
    global _done
    L = lib()
    if not _done:
        for name, (res, args) in _SIGS.items():
            fn = getattr(L, name)
            fn.restype = res
            fn.argtypes = args
        _done = True
    return L


MAX_GATES = 8192
DROP_GATE = 8192


def _valid_gate(g):
    return g < MAX_GATES or g == DROP_GATE


class OracleHashLB:
    """core/modules/hash_lb.{h,cc}"""
    L2, L3, L4, FIELDS = 0, 1, 2, 3
    K_MAX_GATES = 16384  # hash_lb.h kMaxGates

    def __init__(self, gates=(), mode="", fields=()):
        # 115-134
        self.gates_ = [0] * self.K_MAX_GATES
        self.num_gates = 0
        self.mode = self.L4
        self.fields = []          # fields_table_ fields (offset, size)
        self.hash_len = 0         # hasher_(0)
        self._em = None
        self.set_gates(gates=gates)
        if not mode and not fields:
            self.mode = self.L4  # kDefaultMode
            return
        self.set_mode(mode=mode, fields=fields)

    def set_mode(self, mode="", fields=()):
        # 76-98
        if fields:
            self.mode = self.FIELDS
            L = mlib()
            if self._em:
                L.or_em_free(self._em)
            self._em = L.or_em_new()
            self.fields = []
            for i, f in enumerate(fields):
                off = int(f.get("offset", 0)) & 0xFFFFFFFF
                if off >= 1 << 31:
                    off -= 1 << 32  # uint32 -> int
                msg = C.create_string_buffer(256)
                rc = L.or_em_add_field(self._em, off, int(f.get("num_bytes", 0)),
                                       0, i, msg, 256)
                if rc:
                    raise OracleError(rc, "Error adding field %d: %s"
                                      % (i, msg.value.decode()))
                self.fields.append((off, int(f.get("num_bytes", 0))))
            self.hash_len = L.or_em_total_key_size(self._em)
        elif mode == "l2":
            self.mode = self.L2
        elif mode == "l3":
            self.mode = self.L3
        elif mode == "l4":
            self.mode = self.L4
        else:
            raise OracleError(E.EINVAL, "available LB modes: l2, l3, l4")

    def set_gates(self, gates=()):
        # 100-113
        if len(gates) > self.K_MAX_GATES:
            raise OracleError(E.EINVAL, "HashLB can have at most %d ogates"
                              % self.K_MAX_GATES)
        for i, g in enumerate(gates):
            self.gates_[i] = int(g) & 0xFFFF  # gate_idx_t
            if not _valid_gate(self.gates_[i]):
                raise OracleError(E.EINVAL, "Invalid ogate %d" % self.gates_[i])
        self.num_gates = len(gates)

    def get_desc(self):
        # 136-138
        return "%d fields" % len(self.fields)

    def process(self, frames, stride, n):
        out = np.empty(n, np.uint16)
        g = np.array(self.gates_, np.uint16)
        mlib().or_hashlb_process(self.mode, self._em, self.hash_len,
                                 g.ctypes.data, self.num_gates, _ptr(frames),
                                 stride, n, out.ctypes.data)
        return out

    def bench(self, frames, stride, n, threads, reps):
        out = np.empty(n, np.uint16)
        g = np.array(self.gates_, np.uint16)
        return mlib().or_hashlb_bench(self.mode, self._em, self.hash_len,
                                      g.ctypes.data, self.num_gates,
                                      _ptr(frames), stride, n, out.ctypes.data,
                                      threads, reps)

    def __del__(self):
        if getattr(self, "_em", None):
            try:
                lib().or_em_free(self._em)
            except Exception:
                pass
            self._em = None


def ipv4_prefix(prefix):
    """Ipv4Prefix(string) (core/utils/ip.cc:63-79) -> (addr, mask) host
    order; OracleError(EINVAL) where the reference's std::stoi throws"""
    a, m = C.c_uint32(), C.c_uint32()
    if mlib().or_ipv4_prefix(prefix.encode(), C.byref(a), C.byref(m)) < 0:
        raise OracleError(E.EINVAL, "invalid prefix length")
    return a.value, m.value


class OracleACL:
    """core/modules/acl.{h,cc}"""

    def __init__(self, rules=()):
        self.rules = []
        self.add(rules=rules)

    def add(self, rules=()):
        # Init 42-53 (CommandAdd 55-58 calls Init)
        new = []
        for r in rules:
            sa, sm = ipv4_prefix(r.get("src_ip", ""))
            da, dm = ipv4_prefix(r.get("dst_ip", ""))
            new.append((sa, sm, da, dm, int(r.get("src_port", 0)) & 0xFFFF,
                        int(r.get("dst_port", 0)) & 0xFFFF,
                        1 if r.get("drop", False) else 0))
        self.rules.extend(new)

    def clear(self):
        self.rules = []

    def _arr(self):
        arr = (or_acl_rule * max(1, len(self.rules)))()
        for i, r in enumerate(self.rules):
            (arr[i].src_addr, arr[i].src_mask, arr[i].dst_addr, arr[i].dst_mask,
             arr[i].src_port, arr[i].dst_port, arr[i].drop) = r
        return arr

    def process(self, frames, stride, n, igate=0):
        out = np.empty(n, np.uint16)
        arr = self._arr()
        mlib().or_acl_process(arr, len(self.rules), _ptr(frames), stride, n,
                              igate, out.ctypes.data)
        return out

    def bench(self, base, stride, n, threads, reps, igate=0):
        out = np.empty(n, np.uint16)
        arr = self._arr()
        return mlib().or_acl_bench(arr, len(self.rules), base, stride, n, igate,
                                   out.ctypes.data, threads, reps)


class OracleIPLookup:
    """core/modules/ip_lookup.{h,cc} with the rte_lpm (DPDK 19.11) table
    semantics it relies on: an existing (prefix, depth) is updated in place;
    a new rule needs room for max_rules rules, and -- deeper than /24 -- a
    tbl8 group for its /24 block unless one is in use (one group per /24
    block holding deeper rules, recycled when the last one goes)."""

    def __init__(self, max_rules=0, max_tbl8s=0):
        # 54-69
        self.max_rules = max_rules or 1024
        self.max_tbl8s = max_tbl8s or 128
        self.default_gate = DROP_GATE
        self.rules = {}  # (masked ip, depth) -> next hop

    @staticmethod
    def _parse(prefix, prefix_len):
        # 153-184 ParseIpv4Prefix
        if not prefix:
            raise OracleError(E.EINVAL, "prefix' is missing")
        addr = C.c_uint32()
        if not mlib().or_ipv4_address(prefix.encode(), C.byref(addr)):
            raise OracleError(E.EINVAL, "Invalid IP prefix: %s" % prefix)
        a = addr.value
        if prefix_len > 32:
            raise OracleError(E.EINVAL, "Invalid prefix length: %d" % prefix_len)
        mask = 0 if prefix_len == 0 else (0xFFFFFFFF << (32 - prefix_len)) & 0xFFFFFFFF
        if a & ~mask & 0xFFFFFFFF:
            raise OracleError(E.EINVAL, "Invalid IP prefix %s/%d %x %x"
                              % (prefix, prefix_len, a, mask))
        return a

    def _tbl8s_in_use(self):
        return len({ip >> 8 for (ip, d) in self.rules if d > 24})

    def add(self, prefix="", prefix_len=0, gate=0):
        # 186-211
        gate = int(gate) & 0xFFFF
        a = self._parse(prefix, prefix_len)
        if not _valid_gate(gate):
            raise OracleError(E.EINVAL, "Invalid gate: %d" % gate)
        if prefix_len == 0:
            self.default_gate = gate
            return
        key = (a, prefix_len)
        if key not in self.rules:
            if len(self.rules) >= self.max_rules:
                raise OracleError(E.ENOSPC, "rpm_lpm_add() failed")
            if prefix_len > 24 and not any(d > 24 and ip >> 8 == a >> 8
                                           for (ip, d) in self.rules):
                if self._tbl8s_in_use() >= min(self.max_tbl8s, 0x7FFF):
                    raise OracleError(E.ENOSPC, "rpm_lpm_add() failed")
        self.rules[key] = gate

    def delete(self, prefix="", prefix_len=0):
        # 213-233
        a = self._parse(prefix, prefix_len)
        if prefix_len == 0:
            self.default_gate = DROP_GATE
            return
        if (a, prefix_len) not in self.rules:
            raise OracleError(E.EINVAL, "rpm_lpm_delete() failed")
        del self.rules[(a, prefix_len)]

    def clear(self):
        self.rules = {}

    def dir24(self):
        """rte_lpm's DIR-24-8 lookup structure over the current rules (the
        CPU baseline's lookup; or_dir24_free it)"""
        k = list(self.rules.items())
        ips = np.array([x[0][0] for x in k] or [0], np.uint32)
        ds = np.array([x[0][1] for x in k] or [0], np.uint8)
        nh = np.array([x[1] for x in k] or [0], np.uint32)
        return mlib().or_dir24_build(ips.ctypes.data, ds.ctypes.data,
                                     nh.ctypes.data, len(k))

    def process(self, frames, stride, n):
        out = np.empty(n, np.uint16)
        k = list(self.rules.items())
        ips = np.array([x[0][0] for x in k] or [0], np.uint32)
        ds = np.array([x[0][1] for x in k] or [0], np.uint8)
        nh = np.array([x[1] for x in k] or [0], np.uint32)
        mlib().or_lpm_process(ips.ctypes.data, ds.ctypes.data, nh.ctypes.data,
                              len(k), _ptr(frames), stride, n, self.default_gate,
                              out.ctypes.data)
        return out



def update_ttl_process(frames, stride, n):
    """UpdateTTL::ProcessBatch (update_ttl.cc:39-58), in place -> gates"""
    out = np.empty(n, np.uint16)
    mlib().or_update_ttl_process(_ptr(frames), stride, n, out.ctypes.data)
    return out


def _ipv4(s):
    """ParseIpv4Address (core/utils/ip.cc:40-51) -> host-order int or None"""
    a = C.c_uint32()
    return a.value if mlib().or_ipv4_address(s.encode(), C.byref(a)) else None


class OracleStaticNAT:
    """core/modules/static_nat.{h,cc}"""

    def __init__(self, pairs=()):
        # Init 46-90
        self.pairs_ = []
        for p in pairs:
            ir, er = p.get("int_range", {}), p.get("ext_range", {})
            vals = []
            for rng, what in ((ir, "internal"), (er, "external")):
                st, en = rng.get("start", ""), rng.get("end", "")
                a = _ipv4(st)
                if a is None:
                    raise OracleError(E.EINVAL, "invalid IP address %s" % st)
                b = _ipv4(en)
                if b is None:
                    raise OracleError(E.EINVAL, "invalid IP address %s" % en)
                if a > b:
                    raise OracleError(E.EINVAL,
                                      "invalid %s IP address range" % what)
                vals += [a, b]
            is_, ie, es, ee = vals
            if ie == 0xFFFFFFFF or ee == 0xFFFFFFFF:
                raise OracleError(E.EINVAL, "cannot map broadcast address")
            if ie - is_ != ee - es:
                raise OracleError(E.EINVAL,
                                  "internal/external address ranges differ")
            self.pairs_.append((is_, es, ie - is_ + 1))

    def get_initial_arg(self):
        # 92-109: the end reported is start + size (one past the range)
        f = lambda a: "%d.%d.%d.%d" % (a >> 24, (a >> 16) & 255, (a >> 8) & 255,
                                       a & 255)
        return {"pairs": [{"int_range": {"start": f(i), "end": f(i + z)},
                           "ext_range": {"start": f(e), "end": f(e + z)}}
                          for i, e, z in self.pairs_]}

    def bench(self, base, stride, n, threads, reps):
        """forward ProcessBatch timed over `threads` pinned threads (CPU
        baseline); in place; returns seconds"""
        k = self.pairs_ or [(0, 0, 0)]
        self._b = [np.array([x[j] for x in k], np.uint32) for j in range(3)]
        out = np.empty(n, np.uint16)
        return mlib().or_static_nat_bench(
            self._b[0].ctypes.data, self._b[1].ctypes.data, self._b[2].ctypes.data,
            len(self.pairs_), base, stride, n, out.ctypes.data, threads, reps)

    def process(self, frames, stride, n, igate=0):
        """ProcessBatch 179-187 (igate 0 forward, else reverse), in place"""
        k = self.pairs_ or [(0, 0, 0)]
        ia = np.array([x[0] for x in k], np.uint32)
        ea = np.array([x[1] for x in k], np.uint32)
        sz = np.array([x[2] for x in k], np.uint32)
        out = np.empty(n, np.uint16)
        mlib().or_static_nat_process(ia.ctypes.data, ea.ctypes.data,
                                     sz.ctypes.data, len(self.pairs_),
                                     _ptr(frames), stride, n,
                                     0 if igate == 0 else 1, out.ctypes.data)
        return out


def ip_encap_process(slots, stride, n, meta_off, offs, head, length):
    """IPEncap::ProcessBatch (ip_encap.cc:40-80) in place on a slab; offs:
    5 attribute offsets (ip_src, ip_dst, ip_proto, ip_nexthop, ether_type),
    < 0 invalid; head (uint16) / length (uint32) updated -> gates"""
    o = np.ascontiguousarray(offs, np.int32)
    out = np.empty(n, np.uint16)
    mlib().or_ip_encap_process(_ptr(slots), stride, n, meta_off, o.ctypes.data,
                               head.ctypes.data, length.ctypes.data,
                               out.ctypes.data)
    return out


class OracleRewrite:
    """core/modules/rewrite.{h,cc}: Init = add; add / clear; ProcessBatch
    over a slab of packet slots (data at slot + head[i]) in batches of 32."""
    SNBUF_HEADROOM = 128

    def __init__(self, templates=()):
        self.h = mlib().or_rewrite_new()
        self.add(templates)

    def __del__(self):
        if getattr(self, "h", None):
            mlib().or_rewrite_free(self.h)
            self.h = None

    def add(self, templates):
        """templates: bytes objects -> raises ValueError(errno, msg)"""
        k = len(templates)
        bufs = [C.create_string_buffer(bytes(t), max(len(t), 1)) for t in templates]
        ptrs = (C.c_void_p * max(k, 1))(*[C.addressof(b) for b in bufs])
        lens = (C.c_uint32 * max(k, 1))(*[len(t) for t in templates])
        msg = C.create_string_buffer(256)
        r = mlib().or_rewrite_add(self.h, ptrs, lens, k, msg, 256)
        if r:
            raise ValueError(-r, msg.value.decode())

    def clear(self):
        mlib().or_rewrite_clear(self.h)

    def process(self, slots, stride, n, head, length, headroom=SNBUF_HEADROOM):
        mlib().or_rewrite_process(self.h, _ptr(slots), stride, n, headroom,
                                  head.ctypes.data, length.ctypes.data)


class OracleNAT:
    """core/modules/nat.{h,cc}; seed: the module's Random (rdtsc in the
    reference)"""

    def __init__(self, ext_addrs=(), seed=0x5EED):
        # Init 46-96: every range is checked before any address
        for a in ext_addrs:
            for r in a.get("port_ranges", []):
                b, e = int(r.get("begin", 0)), int(r.get("end", 0))
                if b >= e or b > 65535 or e > 65535:
                    raise OracleError(E.EINVAL, "Port range for address %s is "
                                      "malformed" % a.get("ext_addr", ""))
        addrs, nr, beg, end, sus = [], [], [], [], []
        for a in ext_addrs:
            v = _ipv4(a.get("ext_addr", ""))
            if v is None:
                raise OracleError(E.EINVAL, "invalid IP address %s"
                                  % a.get("ext_addr", ""))
            addrs.append(v)
            rl = a.get("port_ranges", [])
            nr.append(len(rl))
            for r in rl:
                beg.append(int(r["begin"]))
                end.append(int(r["end"]))
                sus.append(1 if r.get("suspended", False) else 0)
        if not addrs:
            raise OracleError(E.EINVAL,
                              "at least one external IP address must be specified")
        self.h = mlib().or_nat_new(seed)
        A = np.array(addrs, np.uint32)
        N = np.array(nr, np.uint32)
        B = np.array(beg or [0], np.uint16)
        En = np.array(end or [0], np.uint16)
        S = np.array(sus or [0], np.uint8)
        mlib().or_nat_init(self.h, A.ctypes.data, len(addrs), N.ctypes.data,
                           B.ctypes.data, En.ctypes.data, S.ctypes.data)

    def __del__(self):
        if getattr(self, "h", None):
            mlib().or_nat_free(self.h)
            self.h = None

    def desc(self):
        return "%d entries" % (mlib().or_nat_count(self.h) // 2)

    def process(self, frames, stride, n, igate, now):
        out = np.empty(n, np.uint16)
        mlib().or_nat_process(self.h, _ptr(frames), stride, n,
                              0 if igate == 0 else 1, now, out.ctypes.data)
        return out
