"""WildcardMatch at the reference's full key width.

The reference takes up to 8 fields of 1-8 bytes each (MAX_FIELDS,
MAX_FIELD_SIZE, core/modules/wildcard_match.h:45-51) at offsets 0-1024
(AddFieldOne, wildcard_match.cc:75-100): a key of up to 64 B, which the
device tables hold as KW = 8 u64 words. Round 5's tests never went past a
24 B key. Here 5-8 field keys of 33-64 B run through every WildcardMatch
path, bit-exact against the oracle's WildcardMatch::ProcessBatch /
LookupEntry (wildcard_match.cc:136-203, restated in oracle/oracle.c):

* layouts inside one 64 B window (four 16 B chunks), overlapping fields
  read from a 32 B window (the pair loads), a window past the slot's first
  line, and fields spread over 1 KB (no window: per-field loads; on a
  tag-word image the L2 fallback of bg_kernels.hip launch_wm);
* images: the whole table in LDS, tag words in LDS (the run-time compiled
  kernel and the ahead-of-time one), the key filter, the table in L2;
* entry points: device slabs (bg_wm_classify), staged host windows
  (bg_wm_process_host), the persistent ring (bg_wm_ring_*), and the module
  through its aggregation queue in ring and launch mode (bg_pipe_*);
* priority ties across 8 tuples of 64 B keys (P5: the later tuple wins).

CPU tests: the wide layouts' run-time compiled kernels build for gfx950."""
import numpy as np
import pytest

from bess_amd import _lib as LB
from bess_amd import flowtable as F
from oracle import oracle as O

# (offset, size) per field
LAYOUTS = {
    # 8 x 8 B: the 64 B key, window [0, 64)
    "w64": [(8 * i, 8) for i in range(8)],
    # 5 fields with gaps, 40 B, window [0, 64)
    "w40": [(0, 8), (12, 8), (24, 8), (36, 8), (48, 8)],
    # 33 B: the smallest KW = 8 key, its last byte at 63
    "w33": [(3, 8), (14, 8), (26, 8), (38, 8), (63, 1)],
    # overlapping fields (the reference does not forbid them): a 48 B key
    # out of bytes [0, 18), the two-chunk window the pair loads read
    "ovl": [(0, 8), (2, 8), (4, 8), (6, 8), (8, 8), (10, 8)],
    # 7 fields, 46 B, window [64, 128): past the slot's first line
    "hi": [(68, 8), (78, 6), (84, 8), (94, 8), (104, 8), (114, 6), (124, 2)],
    # 6 fields spread over the first KiB, 43 B: no window (per-field loads)
    "far": [(14, 8), (200, 8), (333, 7), (512, 8), (700, 4), (1016, 8)],
}
SPAN = {k: max(o + s for o, s in v) for k, v in LAYOUTS.items()}


def key_of(frames, fields):
    """the WildcardMatch key bytes of each frame (fields concatenated)"""
    return np.concatenate([frames[:, o:o + s] for o, s in fields], axis=1)


def masks_for(ks, n_masks, rng):
    """n_masks distinct masks over a ks-byte key: one one-byte (partial) mask,
    one two-byte mask (the direct-tuple shapes), the rest covering 40-90 %
    of the key, one of them the whole key"""
    out = []
    while len(out) < n_masks:
        m = np.zeros(ks, np.uint8)
        i = len(out)
        if i == 0:
            m[int(rng.integers(ks))] = 0xF0
        elif i == 1:
            m[rng.choice(ks, 2, replace=False)] = 0xFF
        elif i == 2:
            m[:] = 0xFF
        else:
            m[rng.random(ks) < rng.uniform(0.4, 0.9)] = 0xFF
            m[int(rng.integers(ks))] = 0xFF
        if not any((m == x).all() for x in out):
            out.append(m)
    return out


def workload(fields, n_rules, n_pkts, stride, seed, n_masks=6, prio_range=20):
    """Rules cut from source frames under n_masks masks; packets: a third
    copies of a source frame, a third copies with one key byte changed (only
    the masks that do not cover it still match), a third random"""
    rng = np.random.default_rng(seed)
    ks = sum(s for _, s in fields)
    n_src = max(1, n_rules // 2)
    src = rng.integers(0, 256, (n_src, stride), dtype=np.uint8)
    skey = key_of(src, fields)
    masks = masks_for(ks, n_masks, rng)
    mi = rng.integers(0, n_masks, n_rules)
    mi[:n_masks] = np.arange(n_masks)  # every mask has a rule
    si = rng.integers(0, n_src, n_rules)
    rm = np.stack([masks[i] for i in mi])
    rk = skey[si] & rm
    prio = rng.integers(0, prio_range, n_rules).astype(np.int32)
    gates = rng.integers(0, 64, n_rules).astype(np.uint16)
    frames = rng.integers(0, 256, (n_pkts, stride), dtype=np.uint8)
    kind = rng.integers(0, 3, n_pkts)
    pick = rng.integers(0, n_src, n_pkts)
    frames[kind < 2] = src[pick[kind < 2]]
    # change one field byte of the second third
    chg = np.nonzero(kind == 1)[0]
    flat = [o + j for o, s in fields for j in range(s)]
    at = np.array(flat)[rng.integers(0, len(flat), len(chg))]
    frames[chg, at] ^= rng.integers(1, 256, len(chg), dtype=np.uint8)
    return rk, rm, prio, gates, frames


def oracle_gates(fields, rk, rm, prio, gates, frames, stride, default_gate):
    L = O.lib()
    wm = L.or_wm_new()
    for off, size in fields:
        assert L.or_wm_add_field(wm, off, size, None, 0) == 0
    L.or_wm_init_done(wm)
    kb = np.zeros(64, np.uint8)
    mb = np.zeros(64, np.uint8)
    for k, m, p, g in zip(rk, rm, prio, gates):
        kb[:] = 0
        mb[:] = 0
        kb[:len(k)] = k
        mb[:len(m)] = m
        assert L.or_wm_add(wm, kb.ctypes.data, mb.ctypes.data, int(p), int(g)) == 0
    n = len(frames)
    want = np.zeros(n, np.uint16)
    f = np.ascontiguousarray(frames)
    L.or_wm_process(wm, f.ctypes.data, stride, n, default_gate, want.ctypes.data)
    L.or_wm_free(wm)
    return want


def make_table(fields, rk, rm, prio, gates):
    t = F.WmTable(fields)
    for k, m, p, g in zip(rk, rm, prio, gates):
        t.add(k.tobytes(), m.tobytes(), int(p), int(g))
    return t


def rule_args(fields, k, m, p, g):
    """a module `add` argument (WildcardMatchCommandAddArg) of one rule"""
    vals, msks, pos = [], [], 0
    kb, mb = k.tobytes(), m.tobytes()
    for _, s in fields:
        vals.append({"value_bin": kb[pos:pos + s]})
        msks.append({"value_bin": mb[pos:pos + s]})
        pos += s
    return dict(gate=int(g), priority=int(p), values=vals, masks=msks)


# ------------------------------------------------------------------ CPU
@pytest.mark.parametrize("name", ["w64", "w40", "w33", "ovl", "hi"])
def test_wide_layout_jit_compiles(name):
    """the run-time compiled kernel of a KW = 8 tag-word image builds"""
    fields = LAYOUTS[name]
    rk, rm, prio, gates, _ = workload(fields, 20000, 1, max(64, SPAN[name]), seed=3)
    t = make_table(fields, rk, rm, prio, gates)
    assert 32 < t.key_size <= 64  # KW = 8
    rc, code, log = t.jit_check()
    assert rc == 0, log
    assert code > 4096


def test_far_layout_has_no_window_kernel():
    """fields over 1 KB have no key window: nothing to compile (the
    ahead-of-time per-field kernels serve the image)"""
    import errno
    fields = LAYOUTS["far"]
    rk, rm, prio, gates, _ = workload(fields, 20000, 1, 1024, seed=4)
    t = make_table(fields, rk, rm, prio, gates)
    rc, code, _ = t.jit_check()
    assert rc in (0, -errno.ENOENT)
    if rc:
        assert code == 0


def test_wide_oracle_self_consistent():
    """the workload's rules hit: a third of the packets are their sources"""
    fields = LAYOUTS["w64"]
    rk, rm, prio, gates, frames = workload(fields, 3000, 4000, 64, seed=5)
    want = oracle_gates(fields, rk, rm, prio, gates, frames, 64, 999)
    assert (want != 999).mean() > 0.4


# ------------------------------------------------------------------ GPU
def _torch():
    return pytest.importorskip("torch")


def dev_gates(t, d_frames, stride, n, default_gate, flags):
    torch = _torch()
    d_g = torch.full((n,), -1, dtype=torch.int16, device="cuda")
    with LB.kernel_paths(flags):
        t.classify(d_frames, stride, n, default_gate, d_g)
        torch.cuda.synchronize()
    return d_g.cpu().numpy().view(np.uint16)


def jit_ready(t):
    import errno
    try:
        t.jit_wait(0)
    except LB.BessGpuError as e:
        if e.code == errno.ENOENT:
            return False
        raise
    return True


SMALL_PATHS = (0, LB.BG_PATH_FORCE_LDS, LB.BG_PATH_NO_LDS, LB.BG_PATH_NO_SLAB,
               LB.BG_PATH_NO_SLAB | LB.BG_PATH_FORCE_LDS)
BIG_PATHS = (0, LB.BG_PATH_WM_NO_JIT, LB.BG_PATH_NO_LDS, LB.BG_PATH_NO_SLAB,
             LB.BG_PATH_WM_NO_TAGS, LB.BG_PATH_WM_NO_TAGS | LB.BG_PATH_NO_LDS)


@pytest.mark.gpu
@pytest.mark.parametrize("name,stride", [("w64", 64), ("w40", 64), ("w33", 96),
                                         ("ovl", 64), ("ovl", 2048), ("hi", 128),
                                         ("hi", 2048), ("far", 1024), ("far", 2048)])
@pytest.mark.parametrize("n_rules", [200, 30000])
def test_wide_vs_oracle_every_image(name, stride, n_rules):
    """200 rules: the whole table in LDS (or L2 when forced); 30 K rules: tag
    words in LDS (compiled kernel and not), the key filter, L2. Ragged
    packet counts end in partial tiles."""
    torch = _torch()
    fields = LAYOUTS[name]
    n = 40000 + 37
    rk, rm, prio, gates, frames = workload(fields, n_rules, n, stride, seed=n_rules + stride)
    t = make_table(fields, rk, rm, prio, gates)
    assert 32 < t.key_size <= 64  # KW = 8
    want = oracle_gates(fields, rk, rm, prio, gates, frames, stride, 777)
    d = torch.from_numpy(frames.reshape(-1)).cuda()
    t.sync(0)
    big = n_rules > 1000
    assert t.table_info()[1] == (3 if big else 1)
    if big:
        jit_ready(t)
    for flags in (BIG_PATHS if big else SMALL_PATHS):
        got = dev_gates(t, d, stride, n, 777, flags)
        bad = np.nonzero(got != want)[0]
        assert len(bad) == 0, (name, stride, flags, len(bad), bad[:5], got[bad[:5]], want[bad[:5]])
    assert (want != 777).mean() > 0.3
    # the staged host path: only the fields' window (or bytes) travel
    got = t.process_host(frames, stride, 3001, 777)
    assert (got == want[:3001]).all()


@pytest.mark.gpu
@pytest.mark.parametrize("name,stride", [("w64", 64), ("ovl", 2048), ("far", 2048)])
def test_wide_ring_vs_oracle(name, stride):
    """the persistent WildcardMatch kernel (bg_wm_ring_*) over KW = 8 images:
    30 K rules (tag-word image probed in L2) and 300 (LDS)"""
    torch = _torch()
    fields = LAYOUTS[name]
    n = 1 << 15
    for n_rules in (300, 30000):
        rk, rm, prio, gates, frames = workload(fields, n_rules, n, stride, seed=7 + n_rules)
        want = oracle_gates(fields, rk, rm, prio, gates, frames, stride, 8192)
        t = make_table(fields, rk, rm, prio, gates)
        d = torch.from_numpy(frames.reshape(-1)).cuda()
        ring = F.Ring(t, slots=512)
        try:
            for burst in (32, 100, 4096):
                dg = torch.full((n,), -1, dtype=torch.int16, device="cuda")
                ring.run(d, stride, n, burst, 8192, dg)
                got = dg.cpu().numpy().view(np.uint16)
                assert (got == want).all(), (name, n_rules, burst)
        finally:
            ring.close()


@pytest.mark.gpu
@pytest.mark.parametrize("mode", ["ring", "launch"])
@pytest.mark.parametrize("name", ["w64", "ovl", "hi", "far"])
def test_wide_module_pipe_vs_oracle(name, mode):
    """the WildcardMatch module with 5-8 fields through its aggregation queue
    (snbuf-like host buffers, 32-packet submits), then a rule change"""
    from bess_amd._lib import BG_PATH_PIPE_NO_RING, kernel_paths
    from bess_amd.modules import Pipe, WildcardMatch
    from test_gpu_pipe import run_pipe, snbufs
    fields = LAYOUTS[name]
    stride = 2048
    n = 12000
    rk, rm, prio, gates, frames = workload(fields, 24000, n, stride, seed=31)
    fl = [{"offset": o, "num_bytes": s} for o, s in fields]
    m = WildcardMatch(fields=fl)
    ow = O.OracleWildcardMatch(fields=fl)
    half = len(rk) // 2
    m.set_runtime_config(default_gate=9,
                         rules=[rule_args(fields, *r) for r in
                                zip(rk[:half], rm[:half], prio[:half], gates[:half])])
    ow.set_runtime_config(default_gate=9,
                          rules=[rule_args(fields, *r) for r in
                                 zip(rk[:half], rm[:half], prio[:half], gates[:half])])
    _, heads = snbufs(frames)
    with kernel_paths(BG_PATH_PIPE_NO_RING if mode == "launch" else 0):
        pipe = Pipe(m, batch=1024, depth=4)
        try:
            got = run_pipe(pipe, heads, shuffle_seed=3)
            want = ow.process(frames, stride, n)
            assert (got == want).all()
            for r in zip(rk[half:], rm[half:], prio[half:], gates[half:]):
                a = rule_args(fields, *r)
                m.add(**a)
                ow.add(**a)
            got = run_pipe(pipe, heads)
            want = ow.process(frames, stride, n)
            assert (got == want).all() and (want != 9).mean() > 0.3
        finally:
            pipe.close()
    # the module's synchronous host path too
    got = m.process(frames, stride, 2000)
    assert (got == want[:2000]).all()


@pytest.mark.gpu
@pytest.mark.parametrize("filler", [0, 30000])
@pytest.mark.parametrize("name", ["w64", "far"])
def test_wide_priority_ties_eight_tuples(name, filler):
    """8 tuples of a 64 B (43 B) key, one rule each, all matching the same
    packets at one priority: the last tuple wins (P5, `>=` in LookupEntry,
    wildcard_match.cc:136-157); with one priority higher, that rule wins.
    filler: rules in the wide tuples (a table holds 8 tuples) that make the
    image a tag-word one"""
    torch = _torch()
    fields = LAYOUTS[name]
    stride = 64 if name == "w64" else 1024
    ks = sum(s for _, s in fields)
    rng = np.random.default_rng(41)
    masks = masks_for(ks, 8, rng)
    src = rng.integers(0, 256, (4, stride), dtype=np.uint8)
    # the sources differ in the bytes the one- and two-byte masks cover, so
    # no source matches another's narrow rules
    flat = [o + j for o, s in fields for j in range(s)]
    for p in np.nonzero(masks[0] | masks[1])[0]:
        src[:, flat[p]] = [0x11, 0x22, 0x33, 0x44]
    skey = key_of(src, fields)
    rk, rm, prio, gates = [], [], [], []
    for t_, m in enumerate(masks):  # packet 0's source: all 8 tuples at prio 5
        rk.append(skey[0] & m), rm.append(m), prio.append(5), gates.append(10 + t_)
    for t_, m in enumerate(masks):  # packet 1's source: tuple 3 at prio 6
        rk.append(skey[1] & m), rm.append(m), prio.append(6 if t_ == 3 else 5)
        gates.append(20 + t_)
    for t_, m in enumerate(masks[:5]):  # packet 2's source: first five tuples
        rk.append(skey[2] & m), rm.append(m), prio.append(-3), gates.append(30 + t_)
    if filler:
        fk = rng.integers(0, 256, (filler, ks), dtype=np.uint8)
        fi = rng.integers(2, 8, filler)  # wide masks only: no accidental hits
        for k, i in zip(fk, fi):
            rk.append(k & masks[i]), rm.append(masks[i]), prio.append(9), gates.append(50)
    rk, rm = np.stack(rk), np.stack(rm)
    prio = np.array(prio, np.int32)
    gates = np.array(gates, np.uint16)
    t = make_table(fields, rk, rm, prio, gates)
    assert t.num_tuples() == 8
    frames = np.concatenate([src, rng.integers(0, 256, (60, stride), dtype=np.uint8)])
    frames = np.tile(frames, (1000, 1))  # 64 K packets: the LDS images too
    n = len(frames)
    want = oracle_gates(fields, rk, rm, prio, gates, frames, stride, 100)
    assert list(want[:4]) == [17, 23, 34, 100]
    d = torch.from_numpy(frames.reshape(-1)).cuda()
    t.sync(0)
    big = filler > 0
    assert t.table_info()[1] == (3 if big else 1)
    if big:
        jit_ready(t)
    for flags in (BIG_PATHS if big else SMALL_PATHS):
        got = dev_gates(t, d, stride, n, 100, flags)
        assert (got == want).all(), flags
