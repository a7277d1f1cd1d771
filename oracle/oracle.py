"""TEST INFRASTRUCTURE ONLY -- Python face of the CPU oracle.

ctypes bindings to oracle/liboracle.so (the plain-C restatement of the
reference datapath, oracle/oracle.c) plus a Python restatement of the
reference's module control plane (proto argument -> field / rule bytes,
errors, get_initial_arg / get_runtime_config), operating on pybess-style dict
arguments. Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline
leg may import this module; the product (bess_amd) never does.

Citations are NetSys/bess paths relative to its tree.
"""
import ctypes as C
import errno
import os
import struct
import subprocess

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "liboracle.so")
REF_LIB_PATH = os.path.join(HERE, "_ref", "libref_endian.so")

MAX_GATES = 8192          # core/gate.h:57
DROP_GATE = MAX_GATES     # core/gate.h:58
GATE_NONE = 0xFFFF        # oracle sentinel: packet not emitted (P8)
KEY_BYTES = 64


class OracleError(Exception):
    """CommandFailure(errno, message) (core/message.h:44-53)."""

    def __init__(self, code, msg):
        super().__init__("[errno %d] %s" % (code, msg))
        self.code = code
        self.msg = msg


_lib = None


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            subprocess.check_call(["make", "-s", "-C", HERE, "liboracle.so"])
        L = C.CDLL(LIB_PATH)
        u8p, u16p, sz = C.c_void_p, C.c_void_p, C.c_size_t
        sig = {
            "or_uint64_to_bin": (C.c_int, [C.c_void_p, C.c_uint64, sz, C.c_int]),
            "or_key_hash": (C.c_uint32, [C.c_void_p, sz]),
            "or_em_new": (C.c_void_p, []),
            "or_em_free": (None, [C.c_void_p]),
            "or_em_add_field": (C.c_int, [C.c_void_p, C.c_int, C.c_int,
                                          C.c_uint64, C.c_int, C.c_char_p, sz]),
            "or_em_num_fields": (sz, [C.c_void_p]),
            "or_em_get_field": (None, [C.c_void_p, sz, C.POINTER(C.c_uint64),
                                       C.POINTER(C.c_int), C.POINTER(C.c_int),
                                       C.POINTER(C.c_int)]),
            "or_em_total_key_size": (sz, [C.c_void_p]),
            "or_em_add_rule": (C.c_int, [C.c_void_p, C.c_uint16, C.c_void_p,
                                         C.c_void_p, sz, C.c_char_p, sz]),
            "or_em_add_rules": (C.c_int, [C.c_void_p, C.c_void_p, sz, sz,
                                          C.c_void_p]),
            "or_c1_bench": (C.c_double, [C.c_void_p, C.c_void_p, sz, sz,
                                         C.c_uint16, C.c_uint64, C.c_void_p,
                                         C.c_int, C.c_int,
                                         C.POINTER(C.c_uint64)]),
            "or_em_delete_rule": (C.c_int, [C.c_void_p, C.c_void_p, C.c_void_p,
                                            sz, C.c_char_p, sz]),
            "or_em_clear": (None, [C.c_void_p]),
            "or_em_count": (sz, [C.c_void_p]),
            "or_em_iter": (C.c_int, [C.c_void_p, C.POINTER(sz), C.c_void_p,
                                     C.POINTER(C.c_uint16)]),
            "or_em_process": (None, [C.c_void_p, u8p, sz, sz, C.c_uint16, u16p]),
            "or_em_bind_attr": (None, [C.c_void_p, C.c_int, C.c_int]),
            "or_em_process_meta": (None, [C.c_void_p, u8p, sz, u8p, sz, sz,
                                          C.c_uint16, u16p]),
            "or_em_bench": (C.c_double, [C.c_void_p, u8p, sz, sz, C.c_uint16,
                                         u16p, C.c_int, C.c_int]),
            "or_wm_new": (C.c_void_p, []),
            "or_wm_free": (None, [C.c_void_p]),
            "or_wm_add_field": (C.c_int, [C.c_void_p, C.c_int, C.c_int,
                                          C.c_char_p, sz]),
            "or_wm_init_done": (None, [C.c_void_p]),
            "or_wm_total_key_size": (sz, [C.c_void_p]),
            "or_wm_add": (C.c_int, [C.c_void_p, C.c_void_p, C.c_void_p,
                                    C.c_int32, C.c_uint16]),
            "or_wm_delete": (C.c_int, [C.c_void_p, C.c_void_p, C.c_void_p]),
            "or_wm_clear": (None, [C.c_void_p]),
            "or_wm_num_tuples": (C.c_int, [C.c_void_p]),
            "or_wm_tuple_mask": (None, [C.c_void_p, C.c_int, C.c_void_p]),
            "or_wm_tuple_count": (sz, [C.c_void_p, C.c_int]),
            "or_wm_iter": (C.c_int, [C.c_void_p, C.c_int, C.POINTER(sz),
                                     C.c_void_p, C.POINTER(C.c_int32),
                                     C.POINTER(C.c_uint16)]),
            "or_wm_process": (None, [C.c_void_p, u8p, sz, sz, C.c_uint16, u16p]),
            "or_wm_bind_attr": (None, [C.c_void_p, C.c_int, C.c_int]),
            "or_wm_process_meta": (None, [C.c_void_p, u8p, sz, u8p, sz, sz,
                                          C.c_uint16, u16p]),
            "or_wm_bench": (C.c_double, [C.c_void_p, u8p, sz, sz, C.c_uint16,
                                         u16p, C.c_int, C.c_int]),
            "or_calculate_sum": (C.c_uint32, [C.c_void_p, sz]),
            "or_fold_checksum": (C.c_uint16, [C.c_uint32]),
            "or_generic_checksum": (C.c_uint16, [C.c_void_p, sz]),
            "or_ipv4_checksum": (C.c_uint16, [C.c_void_p]),
            "or_ipv4_verify": (C.c_int, [C.c_void_p]),
            "or_udp_checksum": (C.c_uint16, [C.c_void_p, C.c_void_p]),
            "or_udp_verify": (C.c_int, [C.c_void_p, C.c_void_p]),
            "or_tcp_checksum": (C.c_uint16, [C.c_void_p, C.c_void_p]),
            "or_tcp_verify": (C.c_int, [C.c_void_p, C.c_void_p]),
            "or_update_checksum16": (C.c_uint16, [C.c_uint16, C.c_uint16,
                                                  C.c_uint16]),
            "or_update_checksum32": (C.c_uint16, [C.c_uint16, C.c_uint32,
                                                  C.c_uint32]),
            "or_cksum_process": (None, [u8p, sz, sz, C.c_int, C.c_int, u16p,
                                        u16p]),
            "or_cksum_bench": (C.c_double, [u8p, sz, sz, C.c_int, C.c_int,
                                            u16p, C.c_int, C.c_int]),
            "or_num_cpus": (C.c_int, []),
        }
        for name, (res, args) in sig.items():
            fn = getattr(L, name)
            fn.restype = res
            fn.argtypes = args
        _lib = L
    return _lib


def ref_lib():
    """oracle/_ref/libref_endian.so: the reference's core/utils/endian.cc
    compiled in place (None when it was not built)."""
    if not os.path.exists(REF_LIB_PATH):
        return None
    L = C.CDLL(REF_LIB_PATH)
    L.ref_uint64_to_bin.restype = C.c_int
    L.ref_uint64_to_bin.argtypes = [C.c_void_p, C.c_uint64, C.c_size_t, C.c_int]
    return L


def _ptr(buf):
    """address of a writable buffer (bytearray / numpy array / ctypes)."""
    if hasattr(buf, "ctypes"):
        return buf.ctypes.data
    return C.addressof((C.c_char * len(buf)).from_buffer(buf))


# --------------------------------------------------------------------------
# utils
# --------------------------------------------------------------------------
def uint64_to_bin(val, size, big_endian):
    """endian.cc:36-58 -> (ok, bytes)"""
    b = (C.c_uint8 * 8)()
    ok = lib().or_uint64_to_bin(b, val & 0xFFFFFFFFFFFFFFFF, size,
                                1 if big_endian else 0)
    return bool(ok), bytes(b[:size])


def u64_from_bin(b):
    """bess::utils::Copy(&u64, value_bin, size): raw bytes into a LE u64."""
    if len(b) > 8:
        # the reference overruns a stack u64 here (UB); rejected instead
        raise OracleError(errno.EINVAL, "value_bin longer than 8 bytes")
    return int.from_bytes(bytes(b) + b"\x00" * (8 - len(b)), "little")


def _gate16(g):
    return int(g) & 0xFFFF  # proto uint64 -> gate_idx_t (u16) truncation


def is_valid_gate(g):
    return g < MAX_GATES or g == DROP_GATE


def _fd_kind(fd):
    if "value_bin" in fd:
        return "bin"
    if "value_int" in fd:
        return "int"
    return None


class _MetadataRegistry:
    """Module::AddMetadataAttr (core/module.cc:248-285) for the control
    plane: per-module attribute list; attr fields are carried through the
    configuration surface only (no datapath here)."""

    def __init__(self):
        self.names = []
        self.sizes = {}

    def add(self, name, size):
        if len(self.names) >= 16:          # kMaxAttrsPerModule
            return -errno.ENOSPC
        if not name:
            return -errno.EINVAL
        if size < 1 or size > 32:          # kMetadataAttrMaxSize
            return -errno.EINVAL
        if name in self.sizes:
            return -errno.EEXIST
        self.names.append(name)
        self.sizes[name] = size
        return len(self.names) - 1


# --------------------------------------------------------------------------
# ExactMatch (core/modules/exact_match.cc + core/utils/exact_match_table.h)
# --------------------------------------------------------------------------
class OracleExactMatch:
    def __init__(self, fields=(), masks=()):
        """ExactMatch::Init exact_match.cc:93-119"""
        self.h = lib().or_em_new()
        self.meta = _MetadataRegistry()
        self.attr = {}  # idx -> attr name
        fields = list(fields)
        masks = list(masks)
        self.empty_masks = len(masks) == 0
        if len(fields) != len(masks) and not self.empty_masks:
            raise OracleError(errno.EINVAL,
                              "must provide masks for all fields (or no masks "
                              "for default match on all bits on all fields)")
        for i, f in enumerate(fields):
            self._add_field_one(f, {} if self.empty_masks else masks[i], i)
        self.default_gate = DROP_GATE

    def __del__(self):
        if getattr(self, "h", None):
            lib().or_em_free(self.h)
            self.h = None

    def _add_field_one(self, field, mask, idx):
        """AddFieldOne exact_match.cc:62-91"""
        size = int(field.get("num_bytes", 0))
        k = _fd_kind(mask)
        mask64 = 0
        if k == "int":
            mask64 = int(mask["value_int"]) & 0xFFFFFFFFFFFFFFFF
        elif k == "bin":
            mask64 = u64_from_bin(mask["value_bin"])
        msg = C.create_string_buffer(256)
        if "attr_name" in field:
            # DoAddField attr branch (exact_match_table.h:391-443): host
            # byte order mask, metadata attribute instead of an offset.
            if idx >= 8:
                raise OracleError(errno.EINVAL, "idx %d is not in [0,8)" % idx)
            if size < 1 or size > 8:
                raise OracleError(errno.EINVAL,
                                  "idx %d: 'size' must be in [1,8]" % idx)
            aid = self.meta.add(field["attr_name"], size)
            if aid < 0:
                raise OracleError(-aid, "idx %d: add_metadata_attr() failed" % idx)
            # the C table only knows offset fields: register a placeholder
            # offset field with the LE-converted mask so positions line up
            if mask64 == 0:
                m = (1 << (8 * size)) - 1
            else:
                ok, mb = uint64_to_bin(mask64, size, False)
                if not ok:
                    raise OracleError(errno.EINVAL,
                                      "idx %d: not a valid %d-byte mask" % (idx, size))
                m = int.from_bytes(mb, "big")  # re-encoded BE below
            err = lib().or_em_add_field(self.h, 0, size, m, idx, msg, 256)
            if err:
                raise OracleError(err, msg.value.decode())
            self.attr[idx] = field["attr_name"]
        elif "offset" in field:
            off = int(field["offset"])
            if off >= 1 << 31:
                off -= 1 << 32  # uint32 -> int
            err = lib().or_em_add_field(self.h, off, size, mask64, idx, msg, 256)
            if err:
                raise OracleError(err, msg.value.decode())
        else:
            raise OracleError(errno.EINVAL,
                              "idx %d: must specify 'offset' or 'attr_name'" % idx)

    # -- table views
    def num_fields(self):
        return lib().or_em_num_fields(self.h)

    def field(self, i):
        m = C.c_uint64()
        off, pos, size = C.c_int(), C.c_int(), C.c_int()
        lib().or_em_get_field(self.h, i, C.byref(m), C.byref(off), C.byref(pos),
                              C.byref(size))
        return {"mask": m.value, "offset": off.value, "pos": pos.value,
                "size": size.value, "attr_name": self.attr.get(i)}

    def _rule_fields(self, fields):
        """RuleFieldsFromPb exact_match.cc:251-271"""
        out = []
        for i, fd in enumerate(fields):
            fs = self.field(i)["size"] if i < 8 else 0
            if _fd_kind(fd) == "bin":
                out.append(bytes(fd["value_bin"]))
            else:
                v = int(fd.get("value_int", 0)) & 0xFFFFFFFFFFFFFFFF
                out.append(bytes((v >> (8 * j)) & 0xFF for j in range(fs)))
        return out

    def _call_rule(self, fn, vals, *extra):
        n = len(vals)
        bufs = [C.create_string_buffer(v, max(len(v), 1)) for v in vals]
        ptrs = (C.c_void_p * max(n, 1))(*[C.addressof(b) for b in bufs])
        lens = (C.c_size_t * max(n, 1))(*[len(v) for v in vals])
        msg = C.create_string_buffer(256)
        err = fn(self.h, *extra, ptrs, lens, n, msg, 256)
        if err:
            raise OracleError(err, msg.value.decode())

    def add(self, fields=(), gate=0):
        """CommandAdd -> AddRule exact_match.cc:189-205, 273-281"""
        gate = _gate16(gate)
        if not is_valid_gate(gate):
            raise OracleError(errno.EINVAL, "Invalid gate: %d" % gate)
        if len(fields) == 0:
            raise OracleError(errno.EINVAL, "'fields' must be a list")
        self._call_rule(lib().or_em_add_rule, self._rule_fields(fields), gate)

    def delete(self, fields=()):
        """CommandDelete exact_match.cc:283-300"""
        if len(fields) == 0:
            raise OracleError(errno.EINVAL, "argument must be a list")
        self._call_rule(lib().or_em_delete_rule, self._rule_fields(fields))

    def clear(self):
        lib().or_em_clear(self.h)

    def set_default_gate(self, gate):
        self.default_gate = _gate16(gate)  # unvalidated (307-311)

    def count(self):
        return lib().or_em_count(self.h)

    def get_desc(self):
        return "%d fields, %d rules" % (self.num_fields(), self.count())

    def entries(self):
        cur = C.c_size_t(0)
        key = (C.c_uint8 * KEY_BYTES)()
        g = C.c_uint16()
        while lib().or_em_iter(self.h, C.byref(cur), key, C.byref(g)):
            yield bytes(key), g.value

    def get_initial_arg(self):
        """GetInitialArg exact_match.cc:122-147"""
        r = {"fields": []}
        if not self.empty_masks:
            r["masks"] = []
        for i in range(self.num_fields()):
            f = self.field(i)
            if f["attr_name"] is not None:
                fd = {"attr_name": f["attr_name"], "num_bytes": f["size"]}
            else:
                fd = {"offset": f["offset"], "num_bytes": f["size"]}
            r["fields"].append(fd)
            if not self.empty_masks:
                mb = struct.pack("<Q", f["mask"])[:f["size"]]
                r["masks"].append({"value_bin": mb})
        return r

    def get_runtime_config(self):
        """GetRuntimeConfig exact_match.cc:150-187 (sorted output)"""
        rules = []
        fl = [self.field(i) for i in range(self.num_fields())]
        for key, gate in self.entries():
            rules.append({"gate": gate, "fields": [
                {"value_bin": key[f["pos"]:f["pos"] + f["size"]]} for f in fl]})
        rules.sort(key=lambda r: (r["gate"], [x["value_bin"] for x in r["fields"]]))
        return {"default_gate": self.default_gate, "rules": rules}

    def set_runtime_config(self, default_gate=0, rules=()):
        """SetRuntimeConfig exact_match.cc:210-222"""
        self.default_gate = _gate16(default_gate)
        self.clear()
        for r in rules:
            self.add(fields=r.get("fields", []), gate=r.get("gate", 0))

    def process(self, frames, stride, n, meta_off=None, attr_offsets=None):
        """ExactMatch::ProcessBatch over n frames at frames + i*stride (32-
        packet batches). frames: writable buffer; returns list of gates.
        attr_name fields read packet i's metadata area, taken to sit at
        frames + i*stride + meta_off, at the attribute's metadata offset
        attr_offsets[name] (what the pipeline's allocator assigned)."""
        import numpy as np
        gates = np.zeros(n, dtype=np.uint16)
        fl = [self.field(i) for i in range(self.num_fields())]
        meta = None
        if any(f["attr_name"] is not None for f in fl):
            if meta_off is None or attr_offsets is None:
                raise OracleError(errno.ENOTSUP, "attr_name fields: no metadata")
            for i, f in enumerate(fl):
                if f["attr_name"] is not None:
                    lib().or_em_bind_attr(self.h, i, attr_offsets[f["attr_name"]])
            meta = _ptr(frames) + meta_off
        lib().or_em_process_meta(self.h, _ptr(frames), stride, meta, stride, n,
                                 self.default_gate, gates.ctypes.data)
        return gates


# --------------------------------------------------------------------------
# WildcardMatch (core/modules/wildcard_match.cc)
# --------------------------------------------------------------------------
class OracleWildcardMatch:
    def __init__(self, fields=()):
        """Init wildcard_match.cc:111-134 / AddFieldOne 75-100"""
        self.h = lib().or_wm_new()
        self.meta = _MetadataRegistry()
        self.fields = []
        size_acc = 0
        msg = C.create_string_buffer(256)
        for fd in fields:
            size = int(fd.get("num_bytes", 0))
            f = {"pos": size_acc, "size": size, "attr_name": None, "offset": 0}
            self.fields.append(f)
            if size < 1 or size > 8:
                raise OracleError(errno.EINVAL, "'size' must be 1-8")
            if "offset" in fd:
                off = int(fd["offset"])
                if off >= 1 << 31:
                    off -= 1 << 32
                err = lib().or_wm_add_field(self.h, off, size, msg, 256)
                if err:
                    raise OracleError(err, msg.value.decode())
                f["offset"] = off
            elif "attr_name" in fd:
                aid = self.meta.add(fd["attr_name"], size)
                if aid < 0:
                    raise OracleError(-aid, "add_metadata_attr() failed")
                lib().or_wm_add_field(self.h, 0, size, msg, 256)
                f["attr_name"] = fd["attr_name"]
            else:
                raise OracleError(errno.EINVAL, "specify 'offset' or 'attr'")
            size_acc += size
        lib().or_wm_init_done(self.h)
        self.total_key_size = (size_acc + 7) // 8 * 8
        self.default_gate = DROP_GATE

    def __del__(self):
        if getattr(self, "h", None):
            lib().or_wm_free(self.h)
            self.h = None

    def _extract_key_mask(self, values, masks):
        """ExtractKeyMask wildcard_match.cc:215-276"""
        nf = len(self.fields)
        if len(values) != nf:
            raise OracleError(errno.EINVAL, "must specify %d values" % nf)
        if len(masks) != nf:
            raise OracleError(errno.EINVAL, "must specify %d masks" % nf)
        key = bytearray(KEY_BYTES)
        mask = bytearray(KEY_BYTES)
        for i, f in enumerate(self.fields):
            size, pos = f["size"], f["pos"]

            def conv(fd, what):
                k = _fd_kind(fd)
                if k == "int":
                    ok, b = uint64_to_bin(int(fd["value_int"]), size, True)
                    if not ok:
                        raise OracleError(
                            errno.EINVAL,
                            "idx %d: not a correct %d-byte %s" % (i, size, what))
                    return int.from_bytes(b + b"\x00" * (8 - size), "little")
                if k == "bin":
                    return u64_from_bin(fd["value_bin"])
                return 0

            v = conv(values[i], "value")
            m = conv(masks[i], "mask")
            if v & ~m & 0xFFFFFFFFFFFFFFFF:
                raise OracleError(
                    errno.EINVAL,
                    "idx %d: invalid pair of value 0x%0*x and mask 0x%0*x" %
                    (i, size * 2, v, size * 2, m))
            key[pos:pos + size] = struct.pack("<Q", v)[:size]
            mask[pos:pos + size] = struct.pack("<Q", m)[:size]
        return bytes(key), bytes(mask)

    def add(self, gate=0, priority=0, values=(), masks=()):
        """CommandAdd wildcard_match.cc:317-354"""
        gate = _gate16(gate)
        prio = int(priority) & 0xFFFFFFFF
        if prio >= 1 << 31:
            prio -= 1 << 32  # int64 -> int
        key, mask = self._extract_key_mask(values, masks)
        if not is_valid_gate(gate):
            raise OracleError(errno.EINVAL, "Invalid gate: %d" % gate)
        err = lib().or_wm_add(self.h, key, mask, prio, gate)
        if err == errno.ENOSPC:
            raise OracleError(err, "failed to add a new wildcard pattern")
        if err:
            raise OracleError(err, "failed to add a rule")

    def delete(self, values=(), masks=()):
        """CommandDelete wildcard_match.cc:357-377"""
        key, mask = self._extract_key_mask(values, masks)
        err = lib().or_wm_delete(self.h, key, mask)
        if err:
            raise OracleError(err, "failed to delete a rule")

    def clear(self):
        lib().or_wm_clear(self.h)

    def set_default_gate(self, gate):
        self.default_gate = _gate16(gate)

    def tuples(self):
        out = []
        for t in range(lib().or_wm_num_tuples(self.h)):
            m = (C.c_uint8 * KEY_BYTES)()
            lib().or_wm_tuple_mask(self.h, t, m)
            ents = []
            cur = C.c_size_t(0)
            key = (C.c_uint8 * KEY_BYTES)()
            pr = C.c_int32()
            g = C.c_uint16()
            while lib().or_wm_iter(self.h, t, C.byref(cur), key, C.byref(pr),
                                   C.byref(g)):
                ents.append((bytes(key), pr.value, g.value))
            out.append((bytes(m), ents))
        return out

    def get_desc(self):
        n = sum(len(e) for _, e in self.tuples())
        return "%d fields, %d rules" % (len(self.fields), n)

    def get_initial_arg(self):
        """GetInitialArg wildcard_match.cc:391-405"""
        fl = []
        for f in self.fields:
            if f["attr_name"] is not None:
                fl.append({"attr_name": f["attr_name"], "num_bytes": f["size"]})
            else:
                fl.append({"offset": f["offset"], "num_bytes": f["size"]})
        return {"fields": fl}

    def get_runtime_config(self):
        """GetRuntimeConfig wildcard_match.cc:409-460"""
        rules = []
        for mask, ents in self.tuples():
            for key, prio, gate in ents:
                rules.append({
                    "priority": prio, "gate": gate,
                    "values": [{"value_bin": key[f["pos"]:f["pos"] + f["size"]]}
                               for f in self.fields],
                    "masks": [{"value_bin": mask[f["pos"]:f["pos"] + f["size"]]}
                              for f in self.fields]})
        rules.sort(key=lambda r: (r["priority"], r["gate"],
                                  [x["value_bin"] for x in r["masks"]],
                                  [x["value_bin"] for x in r["values"]]))
        return {"default_gate": self.default_gate, "rules": rules}

    def set_runtime_config(self, default_gate=0, rules=()):
        """SetRuntimeConfig wildcard_match.cc:469-481"""
        self.clear()
        self.default_gate = _gate16(default_gate)
        for r in rules:
            self.add(gate=r.get("gate", 0), priority=r.get("priority", 0),
                     values=r.get("values", []), masks=r.get("masks", []))

    def process(self, frames, stride, n, meta_off=None, attr_offsets=None):
        """WildcardMatch::ProcessBatch (wildcard_match.cc:159-203); attr_name
        fields as in OracleExactMatch.process"""
        import numpy as np
        meta = None
        if any(f["attr_name"] is not None for f in self.fields):
            if meta_off is None or attr_offsets is None:
                raise OracleError(errno.ENOTSUP, "attr_name fields: no metadata")
            for i, f in enumerate(self.fields):
                if f["attr_name"] is not None:
                    lib().or_wm_bind_attr(self.h, i, attr_offsets[f["attr_name"]])
            meta = _ptr(frames) + meta_off
        gates = np.zeros(n, dtype=np.uint16)
        lib().or_wm_process_meta(self.h, _ptr(frames), stride, meta, stride, n,
                                 self.default_gate, gates.ctypes.data)
        return gates


# --------------------------------------------------------------------------
# IPChecksum / L4Checksum
# --------------------------------------------------------------------------
def cksum_process(frames, stride, n, mode, verify):
    """mode 1 = IPChecksum, 2 = L4Checksum, 3 = IPChecksum -> L4Checksum.
    Mutates frames in place; returns (ip_gates, l4_gates) numpy arrays."""
    import numpy as np
    ipg = np.full(n, GATE_NONE, dtype=np.uint16)
    l4g = np.full(n, GATE_NONE, dtype=np.uint16)
    lib().or_cksum_process(_ptr(frames), stride, n, mode, 1 if verify else 0,
                           ipg.ctypes.data, l4g.ctypes.data)
    return ipg, l4g


def emit_packets(gates, connected=None, none=0xFFFF, drop_gate=8192, burst=32):
    """Module::EmitPacket / DropPacket (core/module.h:534-594) for packets
    0..n-1 in order, packet i emitted on gates[i] (`none`: the module never
    emits it): a gate >= the ogate count or not connected drops the packet
    (546-549); otherwise it joins its gate's batch, and a new batch is
    started (Task::AddToRun) when the current one holds kMaxBurst packets.
    connected: set of connected gates (None: every gate < 8192).
    Returns (per-packet gate or drop_gate, [(gate, [idx...])] in AddToRun
    order, [dropped idx...])."""
    out, batches, dead, cur = [], [], [], {}
    for i, g in enumerate(gates):
        g = int(g)
        if g == none:
            out.append(none)
            continue
        ok = g < 8192 if connected is None else g in connected
        if not ok:
            out.append(drop_gate)
            dead.append(i)
            continue
        out.append(g)
        b = cur.get(g)
        if b is None or len(batches[b][1]) >= burst:
            batches.append((g, []))
            cur[g] = len(batches) - 1
            b = cur[g]
        batches[b][1].append(i)
    return out, batches, dead
