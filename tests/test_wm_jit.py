"""Run-time compiled WildcardMatch kernels (bess_amd/csrc/bg_wm_jit.cc).

A tag-word image's tuple data and key plan are compiled into a specialised
copy of the bg_wm_body.h kernel with hiprtc. CPU tests: the generated source
carries the image's constants and compiles for gfx950 (hiprtc needs no
device). GPU tests: the compiled kernel against the oracle
(core/modules/wildcard_match.cc:136-203 restated in oracle/oracle.c) and
against the ahead-of-time kernel, over random field layouts, masks, strides
and ragged counts."""
import errno

import numpy as np
import pytest

from bess_amd import _lib as LB
from bess_amd import flowtable as F
from bess_amd import packets as P
from oracle import oracle as O


def bench_table(n_rules):
    rk, rm, prio, gates, frames, _ = P.wm_workload(n_rules, 256, stride=64,
                                                  sizes=((60, 1),))
    t = F.WmTable(P.FIVE_TUPLE)
    for k, m, p, g in zip(rk, rm, prio, gates):
        t.add(k.tobytes(), m.tobytes(), int(p), int(g))
    return t


def random_layout(rng, span):
    """2-6 non-overlapping fields of 1-8 bytes inside [0, span)"""
    while True:
        nf = int(rng.integers(2, 7))
        sizes = [int(x) for x in rng.integers(1, 9, nf)]
        if sum(sizes) > 24:
            continue
        offs = sorted(int(x) for x in rng.choice(span - 8, nf, replace=False))
        ok = all(offs[i] + sizes[i] <= offs[i + 1] for i in range(nf - 1))
        if ok and offs[-1] + sizes[-1] <= span:
            return list(zip(offs, sizes))


def layout_workload(fields, n_rules, n_pkts, stride, rng):
    """rules over 6 random masks of the layout's key bytes (two of them one-
    and two-byte masks, the direct-tuple shapes); frames of random bytes, half
    carrying a rule's key bytes at the field offsets"""
    ks = sum(s for _, s in fields)
    masks = []
    for i in range(6):
        m = np.zeros(ks, np.uint8)
        if i == 0:
            m[int(rng.integers(ks))] = 0xF0
        elif i == 1:
            m[rng.choice(ks, min(2, ks), replace=False)] = 0xFF
        else:
            m[rng.random(ks) < 0.6] = 0xFF
            m[int(rng.integers(ks))] = 0xFF
        masks.append(m)
    base = rng.integers(0, 256, (n_rules, ks), dtype=np.uint8)
    mi = rng.integers(0, len(masks), n_rules)
    rm = np.stack([masks[i] for i in mi])
    rk = base & rm
    prio = rng.integers(0, 50, n_rules).astype(np.int32)
    gates = rng.integers(0, 64, n_rules).astype(np.uint16)
    frames = rng.integers(0, 256, (n_pkts, stride), dtype=np.uint8)
    src = rng.integers(0, n_rules, n_pkts)
    derived = rng.random(n_pkts) < 0.5
    pos = 0
    for off, size in fields:
        frames[derived, off:off + size] = base[src[derived], pos:pos + size]
        pos += size
    return rk, rm, prio, gates, frames


def make_table(fields, rk, rm, prio, gates):
    t = F.WmTable(fields)
    for k, m, p, g in zip(rk, rm, prio, gates):
        t.add(k.tobytes(), m.tobytes(), int(p), int(g))
    return t


# ------------------------------------------------------------------ CPU
def test_source_carries_the_image_constants():
    t = bench_table(20000)
    src = t.jit_source(-1)
    assert "struct WmJitSpec" in src
    # the 5-tuple in 64 B slots: the pair-load and lane-per-packet variants
    assert "bg_wm_jit_pair" in src and "bg_wm_jit_n2" in src
    assert "bg_wm_jit_n4" not in src and "stream" not in src
    # the /8 destination tuple is direct; the source port's 2.5 K rules
    # are too sparse a two-byte tuple to be (bg_api.cc kDirect2MinEntries)
    assert "ndirect(const WmArgs &) { return 1u; }" in src


def test_compiles_for_gfx950():
    t = bench_table(20000)
    rc, code, log = t.jit_check()
    assert rc == 0, log
    assert code > 4096


def test_small_table_has_nothing_to_compile():
    """a table that fits LDS whole never uses tag words: no specialised kernel"""
    t = bench_table(200)
    rc, code, _ = t.jit_check()
    assert rc == -errno.ENOENT and code == 0


@pytest.mark.parametrize("seed", [1, 2, 3])
def test_random_layouts_compile(seed):
    rng = np.random.default_rng(seed)
    fields = random_layout(rng, 64)
    rk, rm, prio, gates, _ = layout_workload(fields, 8000, 1, 64, rng)
    t = make_table(fields, rk, rm, prio, gates)
    rc, code, log = t.jit_check()
    assert rc == 0, (fields, log)


# ------------------------------------------------------------------ GPU
@pytest.mark.gpu
@pytest.mark.parametrize("seed,stride,n", [(11, 64, 65536), (12, 64, 65536 + 37),
                                           (13, 128, 40000), (14, 2048, 20000),
                                           (15, 64, 45), (16, 96, 30001),
                                           (17, 32, 5001), (18, 48, 7000)])
def test_jit_vs_oracle_random_layouts(seed, stride, n):
    torch = pytest.importorskip("torch")
    rng = np.random.default_rng(seed)
    fields = random_layout(rng, min(stride, 64))
    rk, rm, prio, gates, frames = layout_workload(fields, 30000, n, stride, rng)
    t = make_table(fields, rk, rm, prio, gates)
    t.jit_wait()
    assert t.table_info()[1] == 3  # tag words in LDS
    d_frames = torch.from_numpy(frames.reshape(-1)).cuda()
    outs = []
    for flags in (0, LB.BG_PATH_WM_NO_JIT):
        d_g = torch.zeros(n, dtype=torch.int16, device="cuda")
        with LB.kernel_paths(flags):
            t.classify(d_frames, stride, n, 777, d_g)
            torch.cuda.synchronize()
        outs.append(d_g.cpu().numpy().view(np.uint16))
    L = O.lib()
    wm = L.or_wm_new()
    for off, size in fields:
        assert L.or_wm_add_field(wm, off, size, None, 0) == 0
    L.or_wm_init_done(wm)
    kb = np.zeros(64, np.uint8)
    mb = np.zeros(64, np.uint8)
    for k, m, p, g in zip(rk, rm, prio, gates):
        kb[:len(k)] = k
        mb[:len(m)] = m
        assert L.or_wm_add(wm, kb.ctypes.data, mb.ctypes.data, int(p), int(g)) == 0
    want = np.zeros(n, np.uint16)
    L.or_wm_process(wm, frames.ctypes.data, stride, n, 777, want.ctypes.data)
    L.or_wm_free(wm)
    for o in outs:
        assert (o == want).all(), fields
    assert (want != 777).mean() > 0.2


@pytest.mark.gpu
def test_jit_follows_rule_changes():
    """a new mask makes a new shape (a new compile); until it is ready the
    ahead-of-time kernel serves, and both give the oracle's gates"""
    torch = pytest.importorskip("torch")
    rng = np.random.default_rng(21)
    fields = P.FIVE_TUPLE
    rk, rm, prio, gates, frames, _ = P.wm_workload(30000, 8192, stride=64,
                                                  sizes=((60, 1),), seed=21)
    # seven of the workload's eight masks first (a table holds at most 8)
    m0 = np.frombuffer(P.WM_MASKS[0], np.uint8)
    sel = np.nonzero((rm[:20000] != m0).any(axis=1))[0]
    rk0, rm0, prio0, gates0 = rk[sel], rm[sel], prio[sel], gates[sel]
    t = make_table(fields, rk0, rm0, prio0, gates0)
    assert t.num_tuples() == 7
    t.jit_wait()
    src0 = t.jit_source(0)
    # rules in new masks: the shape changes
    extra_m = np.zeros(16, np.uint8)
    extra_m[5:7] = 0xFF
    extra_m[11:13] = 0xFF
    ek = (rk[20000:] | 0) & extra_m
    for k in ek[:5000]:
        t.add(k.tobytes(), extra_m.tobytes(), 7, 9)
    d_frames = torch.from_numpy(frames.reshape(-1)).cuda()
    d_g = torch.zeros(8192, dtype=torch.int16, device="cuda")
    t.classify(d_frames, 64, 8192, 5, d_g)  # may run before the compile ends
    first = d_g.cpu().numpy().view(np.uint16).copy()
    t.jit_wait()
    assert t.jit_source(0) != src0
    t.classify(d_frames, 64, 8192, 5, d_g)
    torch.cuda.synchronize()
    second = d_g.cpu().numpy().view(np.uint16)
    L = O.lib()
    wm = L.or_wm_new()
    for off, size in fields:
        assert L.or_wm_add_field(wm, off, size, None, 0) == 0
    L.or_wm_init_done(wm)
    kb = np.zeros(64, np.uint8)
    mb = np.zeros(64, np.uint8)
    rules = list(zip(rk0, rm0, prio0, gates0))
    rules += [(k, extra_m, 7, 9) for k in ek[:5000]]
    for k, m, p, g in rules:
        kb[:16] = k
        mb[:16] = m
        assert L.or_wm_add(wm, kb.ctypes.data, mb.ctypes.data, int(p), int(g)) == 0
    want = np.zeros(8192, np.uint16)
    L.or_wm_process(wm, frames.ctypes.data, 64, 8192, 5, want.ctypes.data)
    L.or_wm_free(wm)
    assert (first == want).all() and (second == want).all()
    del rng


@pytest.mark.gpu
def test_exit_while_compiling():
    """a process that syncs a tag-word table (starting its background compile)
    and exits at once ends cleanly: bg_shutdown, registered with Python's
    atexit, waits for the compile before LLVM's static destructors run"""
    import os
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    code = ("import sys; sys.path.insert(0, %r)\n"
            "from bess_amd import flowtable as F, packets as P\n"
            "rk, rm, pr, g, _, _ = P.wm_workload(20000, 64, stride=64, sizes=((60, 1),))\n"
            "t = F.WmTable(P.FIVE_TUPLE)\n"
            "[t.add(k.tobytes(), m.tobytes(), int(p), int(x)) for k, m, p, x in zip(rk, rm, pr, g)]\n"
            "t.sync(0)\n" % root)
    r = subprocess.run([sys.executable, "-c", code], timeout=120, capture_output=True)
    assert r.returncode == 0, r.stderr.decode()[-2000:]


@pytest.mark.parametrize("helper", ["missing", "fails"])
def test_compile_without_a_working_helper(tmp_path, helper):
    """the run-time compile runs in bg_rtc next to the library; with no
    helper there, or one that dies, the compile fails with its reason and
    the process carries on (the tables keep the ahead-of-time kernel)"""
    import os
    import shutil
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    shutil.copy(os.path.join(root, "bess_amd", "libbessgpu.so"), tmp_path / "libbessgpu.so")
    if helper == "fails":
        fake = tmp_path / "bg_rtc"
        fake.write_text("#!/bin/sh\nexec 0<&-\necho dying >&2\nexit 3\n")
        fake.chmod(0o755)
    code = ("import sys, errno; sys.path.insert(0, %r)\n"
            "from bess_amd import _lib\n"
            "_lib.LIB_PATH = %r\n"
            "from bess_amd import flowtable as F, packets as P\n"
            "rk, rm, pr, g, _, _ = P.wm_workload(20000, 64, stride=64, sizes=((60, 1),))\n"
            "t = F.WmTable(P.FIVE_TUPLE)\n"
            "[t.add(k.tobytes(), m.tobytes(), int(p), int(x)) for k, m, p, x in zip(rk, rm, pr, g)]\n"
            "rc, code, log = t.jit_check()\n"
            "print(rc, code, log.replace(chr(10), ' ')[:300])\n"
            % (root, str(tmp_path / "libbessgpu.so")))
    r = subprocess.run([sys.executable, "-c", code], timeout=120, capture_output=True, text=True)
    assert r.returncode == 0, r.stderr[-2000:]
    rc, nbytes, log = r.stdout.split(" ", 2)
    assert int(rc) == -errno.ENOEXEC and int(nbytes) == 0
    assert ("not found" in log) if helper == "missing" else ("exit status 3" in log and "dying" in log)
