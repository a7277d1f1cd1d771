"""The ACL decision tree (bg_acl_api.cc build_tree), checked on the CPU: the
image the classify kernel stages in LDS is fetched through bg_acl_tree and
walked here exactly as bg_acl.hip AclTreeOp walks it (node references, bit
fields, leaf records, first match in a leaf); the gates must equal the
oracle's ordered first-match scan (core/modules/acl.cc:63-95) on the same
packets. The kernel itself is checked on the GPU by tests/test_gpu_acl.py."""
import ctypes as C

import numpy as np
import pytest

from bess_amd import _lib as LB
from bess_amd import packets as P
from oracle import oracle_more as OM
from test_gpu_acl import workload

DROP = 8192


class bg_acl_rule(C.Structure):
    _fields_ = [("src_addr", C.c_uint32), ("src_mask", C.c_uint32),
                ("dst_addr", C.c_uint32), ("dst_mask", C.c_uint32),
                ("src_port", C.c_uint16), ("dst_port", C.c_uint16),
                ("drop", C.c_uint8), ("pad", C.c_uint8 * 3)]


def tree_of(rules):
    """(image, root) for the oracle's parsed rules, or None (no tree)."""
    L = LB.lib()
    h = C.c_void_p()
    LB.check(L.bg_acl_create(C.byref(h)))
    try:
        arr = (bg_acl_rule * max(1, len(rules)))()
        for i, r in enumerate(rules):
            a = arr[i]
            (a.src_addr, a.src_mask, a.dst_addr, a.dst_mask, a.src_port,
             a.dst_port, a.drop) = r
        LB.check(L.bg_acl_add(h, arr, len(rules)))
        words, roots, nt = C.c_size_t(), (C.c_uint32 * 4)(), C.c_int()
        rc = L.bg_acl_tree(h, None, 0, C.byref(words), roots, C.byref(nt))
        if rc == -2:  # ENOENT
            return None
        LB.check(rc)
        img = np.zeros(words.value, np.uint32)
        LB.check(L.bg_acl_tree(h, img.ctypes.data, len(img), C.byref(words),
                               roots, C.byref(nt)))
        assert 1 <= nt.value <= 4
        return img, list(roots)[:nt.value]
    finally:
        L.bg_acl_destroy(h)


def packet_fields(frames, stride):
    f = frames.reshape(-1, stride)
    be32 = lambda o: ((f[:, o].astype(np.uint32) << 24) | (f[:, o + 1].astype(np.uint32) << 16)
                      | (f[:, o + 2].astype(np.uint32) << 8) | f[:, o + 3])
    sip, dip = be32(26), be32(30)
    ihl = (f[:, 14] & 0x0F).astype(np.int64)
    l4 = 14 + 4 * ihl
    rows = np.arange(len(f))

    def be16(o):
        ok = o + 2 <= stride
        oo = np.where(ok, o, 0)
        v = (f[rows, oo].astype(np.uint32) << 8) | f[rows, oo + 1]
        return np.where(ok, v, 0).astype(np.uint32)

    ports = be16(l4) | (be16(l4 + 2) << 16)
    return sip, dip, ports


def walk(img, roots, sip, dip, ports, igate=0):
    """AclTreeOp::decide, vectorised over packets"""
    n = len(sip)
    vals = [sip, dip, ports]
    rec = img.reshape(-1, 4)
    best = np.full(n, 0xFFFFFFFF, np.uint64)
    for root in roots:
        ref = np.full(n, root, np.uint32)
        for _ in range(100):
            inner = (ref >> 31) == 0
            if not inner.any():
                break
            dim = np.minimum((ref >> 25) & 3, 2)
            v = np.choose(dim, vals)
            sh, k = (ref >> 16) & 31, (ref >> 21) & 15
            idx = (ref & 0xFFFF) + ((v >> sh) & ((np.uint32(1) << k) - 1))
            ref = np.where(inner, img[np.where(inner, idx, 0)], ref)
        assert ((ref >> 31) == 1).all(), "walk did not reach leaves"
        off, cnt = (ref & 0xFFFF).astype(np.int64), ((ref >> 16) & 0xFF).astype(np.int64)
        done = np.zeros(n, bool)
        for i in range(int(cnt.max()) if n else 0):
            live = ~done & (i < cnt)
            r = rec[np.where(live, off + i, 0)].astype(np.uint64)
            live &= r[:, 3] < best  # records ascend by rule index
            done |= ~live
            w = r[:, 3]
            slen, dlen = w & 63, (w >> 6) & 63
            pm = np.where((w >> 12) & 1, 0xFFFF, 0) | np.where((w >> 13) & 1, 0xFFFF0000, 0)
            miss = ((((sip ^ r[:, 0]) << slen) >> np.uint64(32)) & 0xFFFFFFFF) | \
                   ((((dip ^ r[:, 1]) << dlen) >> np.uint64(32)) & 0xFFFFFFFF) | \
                   ((ports ^ r[:, 2]) & pm.astype(np.uint64))
            hit = live & (miss == 0)
            best[hit] = w[hit]
            done |= hit
    drop = (best == 0xFFFFFFFF) | (((best >> np.uint64(14)) & 1) == 1)
    return np.where(drop, DROP, igate).astype(np.uint16)


def check_list(rules, frames, stride=64, expect_tree=True):
    o = OM.OracleACL(rules=rules)
    t = tree_of(o.rules)
    if t is None:
        assert not expect_tree, "no tree built"
        return None
    img, roots = t
    assert img.size * 4 <= 112 << 10
    want = o.process(frames, stride, len(frames) // stride if frames.ndim == 1 else len(frames))
    got = walk(img, roots, *packet_fields(frames, stride))
    assert (got == want).all(), np.nonzero(got != want)[0][:10]
    return img


@pytest.mark.parametrize("nrules", [1, 2, 9, 10, 33, 100, 300, 1000, 3000])
def test_tree_vs_oracle(nrules):
    rules, f = workload(nrules, 40000, seed=1000 + nrules)
    img = check_list(rules, f)
    assert img is not None


def test_tree_catch_all_first_and_duplicates():
    rng = np.random.default_rng(7)
    rules, f = workload(200, 20000, seed=5)
    # a catch-all in front: every packet takes it
    check_list([{"drop": True}] + rules, f)
    # duplicates, /0 and /32 prefixes, ports only
    extra = [dict(r) for r in rules[:50]] + [
        {"src_ip": "0.0.0.0/0", "dst_port": 80},
        {"src_port": int(rng.integers(1, 65536)), "drop": True},
        {"dst_ip": "10.0.0.0/8"}, {"dst_ip": "10.0.0.0/8", "drop": True}]
    check_list(rules + extra, f)


def test_tree_ports_and_prefix_edges():
    """packets that sit on prefix and port boundaries"""
    rng = np.random.default_rng(11)
    base = rng.integers(0, 1 << 32, 64, dtype=np.uint64).astype(np.uint32)
    rules = []
    for i, b in enumerate(base):
        ln = int(rng.integers(0, 33))
        ip = "%d.%d.%d.%d" % tuple((int(b) >> s) & 255 for s in (24, 16, 8, 0))
        r = {"src_ip": "%s/%d" % (ip, ln), "drop": bool(i & 1)}
        if i % 3 == 0:
            r["src_port"] = int(b) & 0xFFFF or 1
        if i % 5 == 0:
            r["dst_port"] = (int(b) >> 16) or 1
        rules.append(r)
    n = 8192
    pk = P.random_tuples(n, rng)
    pick = rng.integers(0, len(base), n)
    flip = rng.integers(0, 32, n)
    pk["sip"] = (base[pick] ^ (np.uint32(1) << flip.astype(np.uint32))).astype(np.uint32)
    pk["sport"] = (base[pick] & 0xFFFF).astype(np.uint16)
    pk["dport"] = (base[pick] >> 16).astype(np.uint16)
    check_list(rules, P.build_frames(pk, 60, 64))


def test_no_tree_for_non_prefix_masks_or_huge_lists():
    L = LB.lib()
    r = (0x0A000000, 0xFF00FF00, 0, 0, 0, 0, 0)
    assert tree_of([r]) is None
    assert tree_of([]) is None
    rules, _ = workload(9000, 10, seed=3)
    assert tree_of(OM.OracleACL(rules=rules).rules) is None
    assert L  # loaded
