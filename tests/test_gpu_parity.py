"""Parity of the HIP path (libbessgpu.so) against the CPU oracle.

Marked gpu: runs on a real MI355X. Every comparison is bit-exact (gates,
checksum words, whole frames after in-place checksum writes).
"""
import errno
import ctypes as C

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")

from bess_amd import _lib as LB  # noqa: E402
from bess_amd import flowtable as F  # noqa: E402
from bess_amd import packets as P  # noqa: E402
from oracle import oracle as O  # noqa: E402


@pytest.fixture(scope="module")
def dev():
    assert torch.cuda.is_available(), "gpu tests need a HIP device"
    return torch.device("cuda:0")


def to_dev(a, dev):
    return torch.from_numpy(np.ascontiguousarray(a).reshape(-1)).to(dev)


# kernel paths (bg_set_path_flags): where the table is probed -- its own
# choice (LDS for tables <= 40 KB on launches with >= 4096 packets per
# workgroup, else L2), forced LDS, forced L2 -- and, for dense 64 B slots,
# the coalesced slab kernel (default) or the one-slot-per-lane one
TABLE_PATHS = (0, LB.BG_PATH_FORCE_LDS, LB.BG_PATH_NO_LDS, LB.BG_PATH_NO_SLAB,
               LB.BG_PATH_NO_SLAB | LB.BG_PATH_FORCE_LDS)


def classify_all_paths(t, d_frames, stride, n, default_gate, dev):
    """Gates from every table path; asserts they agree, returns them."""
    outs = []
    for flags in TABLE_PATHS:
        with LB.kernel_paths(flags):
            d_g = torch.zeros(n, dtype=torch.int16, device=dev)
            t.classify(d_frames, stride, n, default_gate, d_g)
            torch.cuda.synchronize()
        outs.append(d_g.cpu().numpy().view(np.uint16))
    for o, flags in zip(outs[1:], TABLE_PATHS[1:]):
        assert (o == outs[0]).all(), flags
    return outs[0]


def oracle_em(fields, keys, gates):
    """fields: [(offset, size, mask)] resolved; keys: (n, key_size) u8."""
    L = O.lib()
    em = L.or_em_new()
    for i, (off, size, mask) in enumerate(fields):
        # or_em_add_field takes the proto-level mask (BE-converted inside);
        # convert the resolved key-order mask back to its BE integer
        mb = int(mask).to_bytes(8, "little")[:size]
        assert L.or_em_add_field(em, off, size, int.from_bytes(mb, "big"), i,
                                 None, 0) == 0
    sizes = [s for _, s, _ in fields]
    pos = np.cumsum([0] + sizes)
    ptrs = (C.c_void_p * len(fields))()
    lens = (C.c_size_t * len(fields))(*sizes)
    keys = np.ascontiguousarray(keys)
    for k, g in zip(keys, gates):
        for j in range(len(fields)):
            ptrs[j] = k.ctypes.data + int(pos[j])
        assert L.or_em_add_rule(em, int(g), ptrs, lens, len(fields), None, 0) == 0
    return em


def em_compare(fields, keys, gates, frames, stride, default_gate, dev):
    n = frames.shape[0]
    t = F.EmTable(fields)
    t.add_many(keys, gates)
    got = classify_all_paths(t, to_dev(frames, dev), stride, n, default_gate,
                             dev)
    em = oracle_em(fields, keys, gates)
    want = np.zeros(n, np.uint16)
    O.lib().or_em_process(em, frames.ctypes.data, stride, n, default_gate,
                          want.ctypes.data)
    O.lib().or_em_free(em)
    return got, want, t


# ------------------------------------------------------------- ExactMatch
def test_em_table_kat(golden, dev):
    for case in golden("em_table_kat.json"):
        if not case["packets"]:
            continue
        fields = []
        for off, size, mask in case["fields"]:
            fields.append((off, size, P.default_mask(size) if mask == 0 else mask))
        pk = [bytes.fromhex(p) for p in case["packets"]]
        frames = np.zeros((len(pk), 64), np.uint8)
        for i, p in enumerate(pk):
            frames[i, :len(p)] = np.frombuffer(p, np.uint8)
        t = F.EmTable(fields)
        for r in case["rules"]:
            t.add(b"".join(bytes.fromhex(v) for v in r["fields"]), r["gate"])
        d_gates = torch.zeros(len(pk), dtype=torch.int16, device=dev)
        t.classify(to_dev(frames, dev), 64, len(pk), case["default"], d_gates)
        got = list(d_gates.cpu().numpy().view(np.uint16))
        assert got == case["expect"], case["name"]
        assert list(t.process_host(frames, 64, len(pk), case["default"])) == \
            case["expect"], case["name"]


@pytest.mark.parametrize("n_rules,n_pkts", [(1, 1000), (1000, 65536),
                                            (100000, 262144)])
def test_em_5tuple_vs_oracle(n_rules, n_pkts, dev):
    keys, gates, frames = P.em_workload(n_rules, n_pkts, seed=n_rules)
    got, want, t = em_compare(P.em_fields_5tuple(), keys, gates, frames, 64,
                              8192, dev)
    assert (got == want).all()
    assert 0.3 < (want != 8192).mean() < 0.7  # the workload really hits
    nbytes, in_lds = t.table_info()
    assert in_lds == (n_rules <= 1000)


@pytest.mark.parametrize("n_pkts", [1, 7, 64, 64 * 8 + 7, 100003, (1 << 20) + 37])
@pytest.mark.parametrize("gate_off", [0, 1, 3])
def test_em_slab_held_gates(n_pkts, gate_off, dev):
    """em_slab_kernel with its table in LDS holds the gates of up to 64
    tiles per wave in LDS and stores them 16 B per lane (bg_kernels.hip):
    ragged packet counts (partial tiles, a partial last 8-gate group) and
    gate arrays not 16 B aligned (2-byte stores) land exactly where the
    oracle's do, and nothing past n is written."""
    keys, gates, frames = P.em_workload(1000, n_pkts, seed=0x5EED)
    t = F.EmTable(P.em_fields_5tuple())
    t.add_many(keys, gates)
    em = oracle_em(P.em_fields_5tuple(), keys, gates)
    want = np.zeros(n_pkts, np.uint16)
    O.lib().or_em_process(em, frames.ctypes.data, 64, n_pkts, 8192, want.ctypes.data)
    O.lib().or_em_free(em)
    d_frames = to_dev(frames, dev)
    for flags in (0, LB.BG_PATH_FORCE_LDS):
        buf = torch.full((n_pkts + gate_off + 16,), 0x5A5A, dtype=torch.int16, device=dev)
        with LB.kernel_paths(flags):
            t.classify(d_frames, 64, n_pkts, 8192, buf[gate_off:gate_off + n_pkts])
            torch.cuda.synchronize()
        out = buf.cpu().numpy().view(np.uint16)
        assert (out[gate_off:gate_off + n_pkts] == want).all(), flags
        assert (out[:gate_off] == 0x5A5A).all() and (out[gate_off + n_pkts:] == 0x5A5A).all()
    nbytes, in_lds = t.table_info()
    assert in_lds


@pytest.mark.parametrize("fields", [
    [(0, 4, 0), (6, 2, 0)],                       # 1 key word
    [(23, 1, 0), (26, 4, 0), (30, 4, 0)],         # 2 words (9 B)
    [(0, 8, 0), (8, 8, 0), (16, 8, 0)],           # 3 -> 4 words
    [(i * 7, 7, 0) for i in range(8)],            # 56 B -> 8 words
    [(2, 2, 0xFFF0), (29, 3, 0x00FF00)],          # masks (key byte order)
    [(0, 2, 0), (1000, 4, 0)],                    # far apart: direct loads
    [(1024, 8, 0)],                               # max offset
])
def test_em_field_layouts(fields, dev):
    rng = np.random.default_rng(len(fields))
    fl = [(o, s, P.default_mask(s) if m == 0 else m) for o, s, m in fields]
    stride = max(64, (max(o + s for o, s, _ in fl) + 15) // 16 * 16)
    n = 20000
    frames = rng.integers(0, 4, (n, stride), dtype=np.uint8)  # small alphabet
    ks = sum(s for _, s, _ in fl)
    # rules: keys of some packets (masked), plus random ones
    keys = []
    for i in rng.choice(n, 300, replace=False):
        kb = b""
        for off, size, mask in fl:
            v = int.from_bytes(frames[i, off:off + size].tobytes(), "little")
            kb += (v & mask).to_bytes(size, "little")
        keys.append(kb)
    keys += [rng.integers(0, 4, ks, dtype=np.uint8).tobytes() for _ in range(100)]
    keys = list(dict.fromkeys(keys))
    karr = np.frombuffer(b"".join(keys), np.uint8).reshape(len(keys), ks)
    gates = rng.integers(0, 8192, len(keys)).astype(np.uint16)
    got, want, _ = em_compare(fl, karr, gates, frames, stride, 8192, dev)
    assert (got == want).all()
    assert (want != 8192).any()


@pytest.mark.parametrize("stride", [80, 128, 192, 2048, 2624])
@pytest.mark.parametrize("fields", [
    [(23, 1, 0), (26, 4, 0), (30, 4, 0), (34, 2, 0), (36, 2, 0)],  # window at 16
    [(0, 6, 0), (12, 2, 0)],                                         # at 0
    [(40, 8, 0), (56, 4, 0)],                                        # at 32
])
def test_em_strided_slots_pair_kernel(fields, stride, dev):
    """Frames in slots wider than 64 B with the key window inside the
    slot's first 64 B: em_pair_kernel (two lanes per slot, one 32 B
    request each, round 5) on the default path, the lane kernel under
    BG_PATH_NO_SLAB -- every table path against the oracle, including a
    last tile of fewer than 64 slots"""
    rng = np.random.default_rng(stride)
    fl = [(o, s, P.default_mask(s) if m == 0 else m) for o, s, m in fields]
    n = 20000 + 37
    frames = rng.integers(0, 4, (n, stride), dtype=np.uint8)
    ks = sum(s for _, s, _ in fl)
    keys = []
    for i in rng.choice(n, 400, replace=False):
        kb = b""
        for off, size, mask in fl:
            v = int.from_bytes(frames[i, off:off + size].tobytes(), "little")
            kb += (v & mask).to_bytes(size, "little")
        keys.append(kb)
    keys = list(dict.fromkeys(keys))
    karr = np.frombuffer(b"".join(keys), np.uint8).reshape(len(keys), ks)
    gates = rng.integers(0, 8192, len(keys)).astype(np.uint16)
    got, want, _ = em_compare(fl, karr, gates, frames, stride, 8192, dev)
    assert (got == want).all()
    assert (want != 8192).any()


def test_em_add_delete_resync(dev):
    keys, gates, frames = P.em_workload(500, 8192, seed=3)
    t = F.EmTable(P.em_fields_5tuple())
    t.add_many(keys, gates)
    d_frames = to_dev(frames, dev)
    d_g = torch.zeros(8192, dtype=torch.int16, device=dev)
    t.classify(d_frames, 64, 8192, 9, d_g)
    for k in keys[:250]:
        t.delete(k.tobytes())
    with pytest.raises(F.BessGpuError):
        t.delete(keys[0].tobytes())
    t.classify(d_frames, 64, 8192, 9, d_g)
    got = d_g.cpu().numpy().view(np.uint16)
    em = oracle_em(P.em_fields_5tuple(), keys[250:], gates[250:])
    want = np.zeros(8192, np.uint16)
    O.lib().or_em_process(em, frames.ctypes.data, 64, 8192, 9, want.ctypes.data)
    O.lib().or_em_free(em)
    assert (got == want).all()
    t.clear()
    t.classify(d_frames, 64, 8192, 9, d_g)
    assert (d_g.cpu().numpy() == 9).all()


def test_em_sharded_build_matches_single(dev):
    """The multi-GPU build path (partitioned images, concatenated as an
    all-gather would) gives the same gates as the single-image build."""
    keys, gates, frames = P.em_workload(20000, 65536, seed=11)
    d_frames = to_dev(frames, dev)
    ref = F.EmTable(P.em_fields_5tuple())
    ref.add_many(keys, gates)
    d_ref = torch.zeros(65536, dtype=torch.int16, device=dev)
    ref.classify(d_frames, 64, 65536, 8192, d_ref)
    for nparts in (2, 8):
        t = F.EmTable(P.em_fields_5tuple())
        t.add_many(keys, gates)
        pb = t.plan(nparts)
        img = np.concatenate([t.build_part(p, pb) for p in range(nparts)])
        d_img = to_dev(img, dev)
        t.attach(0, d_img)
        d_g = torch.zeros(65536, dtype=torch.int16, device=dev)
        t.classify(d_frames, 64, 65536, 8192, d_g)
        assert torch.equal(d_g, d_ref)


# ---------------------------------------------------------- WildcardMatch
def classify_all_paths_wm(t, d_frames, stride, n, default_gate, dev, tags):
    """classify_all_paths with BG_PATH_WM_NO_TAGS kept on (tags == 0)"""
    keep = 0 if tags else LB.BG_PATH_WM_NO_TAGS
    paths = TABLE_PATHS
    if tags and wm_jit_ready(t):  # the run-time compiled kernel, then without it
        paths = paths + (LB.BG_PATH_WM_NO_JIT,)
    outs = []
    for flags in paths:
        with LB.kernel_paths(flags | keep):
            d_g = torch.zeros(n, dtype=torch.int16, device=dev)
            t.classify(d_frames, stride, n, default_gate, d_g)
            torch.cuda.synchronize()
        outs.append(d_g.cpu().numpy().view(np.uint16))
    for o, flags in zip(outs[1:], paths[1:]):
        assert (o == outs[0]).all(), flags
    return outs[0]


def wm_jit_ready(t, dev=0):
    """Wait for the table's run-time compiled kernel (bg_wm_jit_wait): True
    once it serves launches, False for an image without tag words."""
    try:
        t.jit_wait(dev)
    except LB.BessGpuError as e:
        if e.code == errno.ENOENT:
            return False
        raise
    return True


def oracle_wm(fields, rkeys, rmasks, prio, gates):
    L = O.lib()
    wm = L.or_wm_new()
    for off, size in fields:
        assert L.or_wm_add_field(wm, off, size, None, 0) == 0
    L.or_wm_init_done(wm)
    kb = np.zeros(64, np.uint8)
    mb = np.zeros(64, np.uint8)
    for k, m, p, g in zip(rkeys, rmasks, prio, gates):
        kb[:len(k)] = k
        mb[:len(m)] = m
        assert L.or_wm_add(wm, kb.ctypes.data, mb.ctypes.data, int(p), int(g)) == 0
    return wm


def test_wm_module_kat(golden, dev):
    for case in golden("wm_module_kat.json"):
        f = [(x["offset"], x["num_bytes"]) for x in case["arg"]["fields"]]
        t = F.WmTable(f)
        dg = 8192
        for cmd, arg in case["cmds"]:
            if cmd == "add":
                k = b"".join(bytes.fromhex(v["value_bin"]) for v in arg["values"])
                m = b"".join(bytes.fromhex(v["value_bin"]) for v in arg["masks"])
                t.add(k, m, arg["priority"], arg["gate"])
            elif cmd == "set_default_gate":
                dg = arg["gate"]
        pk = [bytes.fromhex(p) for p in case["packets"]]
        frames = np.zeros((len(pk), 64), np.uint8)
        for i, p in enumerate(pk):
            frames[i, :] = np.frombuffer(p[:64].ljust(64, b"\0"), np.uint8)
        d_g = torch.zeros(len(pk), dtype=torch.int16, device=dev)
        t.classify(to_dev(frames, dev), 64, len(pk), dg, d_g)
        assert list(d_g.cpu().numpy().view(np.uint16)) == case["expect"]


@pytest.mark.parametrize("n_rules,n_pkts,tags", [
    (64, 4096, 1), (5000, 65536, 1), (5000, 65536, 0), (100000, 131072, 1),
    (100000, 131072, 0), (100000, 131051, 1), (100000, 45, 1), (300000, 65536, 1)])
def test_wm_vs_oracle(n_rules, n_pkts, tags, dev):
    """tags 1: tables past the whole-table LDS size keep their tag words in
    LDS (bg_wm.hip) when they fit; 0 (BG_PATH_WM_NO_TAGS): the key-filter
    path; 300 K rules: tags too big for LDS, the key-filter path either way.
    Ragged counts end in a partial tile (the 64 B slab's pair loads, bg_wm.hip)"""
    rk, rm, prio, gates, frames, _ = P.wm_workload(n_rules, n_pkts,
                                                  seed=n_rules, stride=64,
                                                  sizes=((60, 1),))
    t = F.WmTable(P.FIVE_TUPLE)
    for k, m, p, g in zip(rk, rm, prio, gates):
        t.add(k.tobytes(), m.tobytes(), int(p), int(g))
    assert t.num_tuples() == 8
    with LB.kernel_paths(0 if tags else LB.BG_PATH_WM_NO_TAGS):
        got = classify_all_paths_wm(t, to_dev(frames, dev), 64, n_pkts, 77,
                                    dev, tags)
    wm = oracle_wm(P.FIVE_TUPLE, rk, rm, prio, gates)
    want = np.zeros(n_pkts, np.uint16)
    O.lib().or_wm_process(wm, frames.ctypes.data, 64, n_pkts, 77,
                          want.ctypes.data)
    O.lib().or_wm_free(wm)
    assert (got == want).all()
    assert (want != 77).mean() > 0.3


@pytest.mark.parametrize("n_rules", [100000, 200000])
@pytest.mark.parametrize("n_pkts", [1, 7, 64 * 16 + 9, (1 << 20) + 37])
@pytest.mark.parametrize("gate_off", [0, 1])
def test_wm_tags_held_gates(n_rules, n_pkts, gate_off, dev):
    """the tag-word kernels hold each wave's gates of up to 8 tiles in LDS
    when the CU's LDS has room after the tag words (wm_hold_tiles) and store
    them 16 B per lane: ragged counts, gate arrays not 16 B aligned, both
    WildcardMatch forms (run-time compiled and ahead of time), and nothing
    written outside [0, n)"""
    rk, rm, prio, gates, frames, _ = P.wm_workload(n_rules, n_pkts, seed=n_rules + 7,
                                                  stride=64, sizes=((60, 1),))
    t = F.WmTable(P.FIVE_TUPLE)
    for k, m, p, g in zip(rk, rm, prio, gates):
        t.add(k.tobytes(), m.tobytes(), int(p), int(g))
    wm = oracle_wm(P.FIVE_TUPLE, rk, rm, prio, gates)
    want = np.zeros(n_pkts, np.uint16)
    O.lib().or_wm_process(wm, frames.ctypes.data, 64, n_pkts, 77, want.ctypes.data)
    O.lib().or_wm_free(wm)
    d_frames = to_dev(frames, dev)
    wm_jit_ready(t)
    for flags in (0, LB.BG_PATH_WM_NO_JIT):
        buf = torch.full((n_pkts + gate_off + 16,), 0x5A5A, dtype=torch.int16, device=dev)
        with LB.kernel_paths(flags):
            t.classify(d_frames, 64, n_pkts, 77, buf[gate_off:gate_off + n_pkts])
            torch.cuda.synchronize()
        out = buf.cpu().numpy().view(np.uint16)
        assert (out[gate_off:gate_off + n_pkts] == want).all(), flags
        assert (out[:gate_off] == 0x5A5A).all() and (out[gate_off + n_pkts:] == 0x5A5A).all()


def test_wm_direct_tuples_vs_oracle(dev):
    """Tuples whose masks cover one or two key bytes -- whole and partial
    bytes -- are direct tuples of the tag-word image (bg_wm.hip, WmArgs::
    ndirect; two at most, the rest hashed), mixed with hashed tuples under
    frequent priority ties; then a third of the direct tuples' rules are
    deleted and the image resynced. Every table path, against the oracle."""
    masks = [P._m(proto=0x0F), P._m(sport=0xFF00), P._m(dip=0xFF000000),
             P._m(dport=0xFFF0), P._m(sip=0xFFFFFFFF, dport=0xFFFF),
             P._m(sip=0xFFFF0000, dip=0xFFFF0000), P._m(sport=0xFFFF)]
    n = 65536
    rk, rm, prio, gates, frames, _ = P.wm_workload(60000, n, seed=77, stride=64,
                                                  sizes=((60, 1),), prio_range=20,
                                                  masks=masks)
    t = F.WmTable(P.FIVE_TUPLE)
    for k, m, p, g in zip(rk, rm, prio, gates):
        t.add(k.tobytes(), m.tobytes(), int(p), int(g))
    d_frames = to_dev(frames, dev)

    order = {}  # tuple order: each mask's first add (deletes keep tuples)
    for m in rm:
        order.setdefault(m.tobytes(), len(order))

    def check(keep):
        got = classify_all_paths_wm(t, d_frames, 64, n, 77, dev, 1)
        # the oracle gets the kept rules, each mask's first kept rule added
        # up front in the table's tuple order (equal priorities go to the
        # later tuple, P5), then all of them in order (the later add of a
        # (mask, key) wins, as in the table)
        idx = np.nonzero(keep)[0]
        first = {}
        for i in idx:
            first.setdefault(rm[i].tobytes(), i)
        lead = [first[m] for m in sorted(first, key=order.get)]
        sel = np.concatenate([np.array(lead, np.int64), idx])
        wm = oracle_wm(P.FIVE_TUPLE, rk[sel], rm[sel], prio[sel], gates[sel])
        want = np.zeros(n, np.uint16)
        O.lib().or_wm_process(wm, frames.ctypes.data, 64, n, 77, want.ctypes.data)
        O.lib().or_wm_free(wm)
        assert (got == want).all()
        return want

    want = check(np.ones(len(rk), bool))
    assert t.table_info()[1] == 3 and t.direct_tuples() == 2
    assert (want != 77).mean() > 0.5
    # delete a third of the one- and two-byte tuples' (mask, key) entries
    rng = np.random.default_rng(5)
    few = np.array([np.count_nonzero(m) <= 2 for m in rm])
    pairs = {(k.tobytes(), m.tobytes()) for k, m in zip(rk[few], rm[few])}
    gone = {x for x in sorted(pairs) if rng.random() < 1 / 3}
    for k, m in gone:
        t.delete(k, m)
    keep = np.array([(k.tobytes(), m.tobytes()) not in gone for k, m in zip(rk, rm)])
    check(keep)


def test_wm_dense_two_byte_direct_tuple(dev):
    """A two-byte tuple goes direct (a 65536-entry table read once per
    packet) only when at least half its keys are rules (bg_api.cc
    kDirect2MinEntries); a sparser one is hashed. Both, against the oracle,
    every table path."""
    # the source-port tuple's distinct keys: 34.9 K of 65536 (direct), 9.4 K (hashed)
    for nrules, nd in ((150000, 1), (30000, 0)):
        masks = [P._m(sport=0xFFFF), P._m(sip=0xFFFFFFFF, dport=0xFFFF),
                 P._m(sip=0xFFFF0000, dip=0xFFFF0000)]
        n = 65536
        rk, rm, prio, gates, frames, _ = P.wm_workload(nrules, n, seed=93, stride=64,
                                                      sizes=((60, 1),), masks=masks)
        t = F.WmTable(P.FIVE_TUPLE)
        for k, m, p, g in zip(rk, rm, prio, gates):
            t.add(k.tobytes(), m.tobytes(), int(p), int(g))
        got = classify_all_paths_wm(t, to_dev(frames, dev), 64, n, 77, dev, 1)
        assert t.table_info()[1] == 3 and t.direct_tuples() == nd, nrules
        wm = oracle_wm(P.FIVE_TUPLE, rk, rm, prio, gates)
        want = np.zeros(n, np.uint16)
        O.lib().or_wm_process(wm, frames.ctypes.data, 64, n, 77, want.ctypes.data)
        O.lib().or_wm_free(wm)
        assert (got == want).all(), nrules


@pytest.mark.parametrize("ndirect", [0, 1])
def test_wm_tags_fewer_direct_tuples(dev, ndirect):
    """Tag-word images with no or one direct tuple (masks of three bytes and
    more, or one one-byte mask): a direct slot left unused must not match
    (round 5: its all-ones "empty" value named tuple 0xFFFF, which is what
    an unused slot carried, so every packet without a hit got gate 0xFFFF
    instead of the default gate)"""
    masks = [P._m(sip=0xFFFFFFFF, dport=0xFFFF), P._m(sip=0xFFFF0000, dip=0xFFFF0000),
             P._m(dip=0xFFFFFF00), P._m(proto=0xFF, sport=0xFFFF, dport=0xFFFF)]
    if ndirect:
        masks.append(P._m(dip=0xFF000000))
    n = 65536
    rk, rm, prio, gates, frames, _ = P.wm_workload(40000, n, seed=91, stride=64,
                                                  sizes=((60, 1),), masks=masks)
    t = F.WmTable(P.FIVE_TUPLE)
    for k, m, p, g in zip(rk, rm, prio, gates):
        t.add(k.tobytes(), m.tobytes(), int(p), int(g))
    got = classify_all_paths_wm(t, to_dev(frames, dev), 64, n, 77, dev, 1)
    assert t.table_info()[1] == 3 and t.direct_tuples() == ndirect
    wm = oracle_wm(P.FIVE_TUPLE, rk, rm, prio, gates)
    want = np.zeros(n, np.uint16)
    O.lib().or_wm_process(wm, frames.ctypes.data, 64, n, 77, want.ctypes.data)
    O.lib().or_wm_free(wm)
    assert (got == want).all()
    if ndirect == 0:  # (the /8 tuple's 8 K rules cover every packet)
        assert 0.05 < (want == 77).mean() < 0.95


@pytest.mark.parametrize("filler", [0, 5000])
def test_wm_priority_ties(dev, filler):
    """filler: extra rules in the third tuple make the table too big for
    LDS, so the tag-words-in-LDS kernel (bg_wm.hip) resolves the ties"""
    f = [(0, 1), (1, 1)]
    t = F.WmTable(f)
    t.add(b"\x01\x00", b"\xff\x00", 5, 1)
    t.add(b"\x00\x02", b"\x00\xff", 5, 2)   # later tuple, same prio: wins
    t.add(b"\x01\x02", b"\xff\xff", 4, 3)   # lower prio: loses
    rng = np.random.default_rng(7)
    for v in rng.choice(np.arange(0x2000, 0xFF00), filler, replace=False):
        t.add(int(v).to_bytes(2, "little"), b"\xff\xff", 9, 4)
    frames = np.zeros((4, 64), np.uint8)
    frames[0, :2] = [1, 2]
    frames[1, :2] = [1, 9]
    frames[2, :2] = [9, 2]
    frames[3, :2] = [9, 9]
    d_g = torch.zeros(4, dtype=torch.int16, device=dev)
    t.classify(to_dev(frames, dev), 64, 4, 100, d_g)
    assert list(d_g.cpu().numpy()) == [2, 1, 2, 100]
    # the emptied tuple is only erased by a failing delete (P6)
    t.delete(b"\x00\x02", b"\x00\xff")
    assert t.num_tuples() == 3
    t.delete(b"\x00\x07", b"\x00\xff")
    assert t.num_tuples() == 2
    t.classify(to_dev(frames, dev), 64, 4, 100, d_g)
    assert list(d_g.cpu().numpy()) == [1, 1, 100, 100]


# ------------------------------------------------------------- checksums
def cksum_compare(frames, stride, mode, verify, dev):
    n = frames.shape[0]
    ref = frames.copy()
    ipg_w, l4g_w = O.cksum_process(ref, stride, n, mode, verify)
    d = to_dev(frames, dev)
    ipg = torch.zeros(n, dtype=torch.int16, device=dev)
    l4g = torch.zeros(n, dtype=torch.int16, device=dev)
    F.cksum(d, stride, n, mode, verify, ipg, l4g)
    torch.cuda.synchronize()
    out = d.cpu().numpy().reshape(n, stride)
    return (out, ipg.cpu().numpy().view(np.uint16),
            l4g.cpu().numpy().view(np.uint16), ref, ipg_w, l4g_w)


def edge_frames():
    """Frames for every branch of IPChecksum / L4Checksum (P8-P11)."""
    rng = np.random.default_rng(5)
    t = P.random_tuples(64, rng)
    out = []
    for i, L in enumerate([60, 61, 64, 65, 127, 128, 129, 1496, 1514, 2000]):
        for proto in (6, 17):
            tt = {k: v[i:i + 1].copy() for k, v in t.items()}
            tt["proto"][:] = proto
            f = P.build_frames(tt, L, 2048, rng=rng, payload="random",
                               ip_csum="random")[0]
            out.append(f)
    base = out[0].copy()
    # VLAN and QinQ framed IPv4 (IPChecksum parses them, L4 forwards)
    v = np.zeros(2048, np.uint8)
    v[:12] = base[:12]
    v[12:14] = [0x81, 0x00]
    v[14:16] = [0, 6]
    v[16:2048] = base[12:2044]
    out.append(v)
    q = np.zeros(2048, np.uint8)
    q[:12] = base[:12]
    q[12:14] = [0x88, 0xa8]
    q[14:16] = [0, 5]
    q[16:18] = [0x81, 0x00]
    q[18:20] = [0, 6]
    q[20:2048] = base[12:2040]
    out.append(q)
    q2 = q.copy()
    q2[16:18] = [0x08, 0x00]  # QinQ not followed by 802.1Q: forwarded
    out.append(q2)
    nonip = base.copy()
    nonip[12:14] = [0x86, 0xdd]
    out.append(nonip)
    for src in (2, 3):  # TCP and UDP frames
        for ihl in (0, 1, 2, 3, 4, 6, 15):  # IHL < 5 (L4 overlaps IP) and options
            x = out[src].copy()
            x[14] = 0x40 | ihl
            if src == 3 and ihl > 0:
                # keep the UDP length (now at 18 + 4*ihl) inside the slot:
                # past the 2 KB buffer the reference reads out of bounds (UB)
                at = 18 + 4 * ihl
                if at == 22:
                    x[22] = 0x01  # ttl; with proto 0x11 -> length 0x0111
                else:
                    x[at:at + 2] = [0x01, 0x00]  # 256
            out.append(x)
    icmp = base.copy()
    icmp[23] = 1
    out.append(icmp)
    for ulen in (0, 7, 8, 9):  # UDP length edge cases
        x = out[3].copy()
        x[38:40] = [ulen >> 8, ulen & 0xFF]
        out.append(x)
    for iplen in (39, 40, 20, 0):  # TCP: ip_len < IHL*4 + 20
        x = out[2].copy()
        x[16:18] = [iplen >> 8, iplen & 0xFF]
        out.append(x)
    ones = out[15].copy()
    ones[42:1510] = 0xFF  # all-ones payload (end-around carry)
    out.append(ones)
    zero_ck = out[3].copy()
    zero_ck[40:42] = 0  # UDP checksum 0: verify passes
    out.append(zero_ck)
    return np.stack(out)


@pytest.mark.parametrize("mode", [1, 2, 3])
@pytest.mark.parametrize("verify", [False, True])
def test_cksum_edges_vs_oracle(mode, verify, dev):
    frames = edge_frames()
    # verify mode: make half the frames carry correct checksums first
    if verify:
        O.cksum_process(frames[::2], 2048, frames[::2].shape[0], 3, False)
    out, ipg, l4g, ref, ipw, l4w = cksum_compare(frames, 2048, mode, verify, dev)
    if mode & 1:
        assert (ipg == ipw).all(), np.nonzero(ipg != ipw)
    if mode & 2:
        assert (l4g == l4w).all(), np.nonzero(l4g != l4w)
    assert (out == ref).all(), np.nonzero((out != ref).any(axis=1))


def test_ip_checksum_module_kat(golden, dev):
    k = golden("ip_checksum_module_kat.json")
    frames = np.zeros((len(k["cases"]), 2048), np.uint8)
    for i, c in enumerate(k["cases"]):
        p = bytes.fromhex(c["in"])
        frames[i, :len(p)] = np.frombuffer(p, np.uint8)
    out, ipg, _, _, _, _ = cksum_compare(frames, 2048, 1, False, dev)
    for i, c in enumerate(k["cases"]):
        exp = bytes.fromhex(c["out"])
        assert out[i, :len(exp)].tobytes() == exp, c["name"]
        assert ipg[i] == c["gate"]


@pytest.mark.parametrize("frame_len", [60, 590, 1496])
def test_cksum_workload_vs_oracle(frame_len, dev):
    frames = P.cksum_workload(8192, frame_len=frame_len, seed=frame_len)
    for mode, verify in ((3, False), (2, True), (1, True)):
        out, ipg, l4g, ref, ipw, l4w = cksum_compare(frames.copy(), 2048, mode,
                                                     verify, dev)
        assert (out == ref).all()
        assert (ipg == ipw).all() and (l4g == l4w).all()


def test_host_paths(dev):
    keys, gates, frames = P.em_workload(1000, 4096, seed=9)
    t = F.EmTable(P.em_fields_5tuple())
    t.add_many(keys, gates)
    em = oracle_em(P.em_fields_5tuple(), keys, gates)
    want = np.zeros(4096, np.uint16)
    O.lib().or_em_process(em, frames.ctypes.data, 64, 4096, 8192,
                          want.ctypes.data)
    O.lib().or_em_free(em)
    assert (t.process_host(frames, 64, 4096, 8192) == want).all()
    fr = P.cksum_workload(512, frame_len=1496)
    ref = fr.copy()
    ipw, l4w = O.cksum_process(ref, 2048, 512, 3, False)
    ipg, l4g = F.cksum_host(fr, 2048, 512, 3, False)
    assert (fr == ref).all() and (l4g == l4w).all() and (ipg == ipw).all()
