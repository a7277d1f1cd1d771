"""StaticNAT (core/modules/static_nat.cc): Init validation and
get_initial_arg of the module surface against the oracle; the oracle pinned
the way the reference pins incremental checksum updates
(checksum_test.cc:378-457: after UpdateChecksum32 the full checksum must
verify); the GPU kernel bit-exact against the oracle on random headers in
both directions, every IHL, UDP checksum 0, non-TCP/UDP protocols and
overlapping address pairs (the first pair wins)."""
import errno

import numpy as np
import pytest

from bess_amd import packets as P
from oracle import oracle as O
from oracle import oracle_more as OM


def ip(x):
    return "%d.%d.%d.%d" % ((x >> 24) & 255, (x >> 16) & 255, (x >> 8) & 255, x & 255)


def pair(i0, e0, size):
    return {"int_range": {"start": ip(i0), "end": ip(i0 + size - 1)},
            "ext_range": {"start": ip(e0), "end": ip(e0 + size - 1)}}


# overlapping internal ranges (first pair wins), size-1 ranges, a /8
PAIRS = [pair(0xC0A80100, 0x01020300, 256),
         pair(0xC0A80180, 0x05050500, 128),
         pair(0x0A000000, 0x0B000000, 1 << 24),
         pair(0xAC100001, 0xCB007107, 1),
         pair(0x00000000, 0xFFFFFF00, 16),
         pair(0xFFFFFF00, 0x00000100, 255)]


def nat_frames(n, stride, seed, valid=True, ihl_max=15):
    """IPv4 frames with sources / destinations drawn from both sides of
    PAIRS (and outside them), random IHL 5..ihl_max, TCP / UDP / others,
    some UDP checksums 0. valid: checksums made correct first."""
    rng = np.random.default_rng(seed)
    fl = min(stride, 1496) - 4 if stride > 64 else 60
    f = P.cksum_workload(n, frame_len=fl, stride=stride, seed=seed)
    cands = []
    for p in PAIRS:
        for rng_ in (p["int_range"], p["ext_range"]):
            a = OM._ipv4(rng_["start"])
            b = OM._ipv4(rng_["end"])
            cands += [a, b, (a + b) // 2, a - 1, b + 1]
    cands = np.array([c & 0xFFFFFFFF for c in cands], np.uint64)
    for off in (26, 30):
        pick = rng.random(n) < 0.7
        v = np.where(pick, cands[rng.integers(len(cands), size=n)],
                     rng.integers(0, 1 << 32, n, dtype=np.uint64)).astype(">u4")
        f[:, off:off + 4] = v.view(np.uint8).reshape(n, 4)
    ihl = np.where(rng.random(n) < 0.6, 5, rng.integers(5, ihl_max + 1, n))
    f[:, 14] = (0x40 | ihl).astype(np.uint8)
    # TCP / UDP as built (lengths consistent), 20 % other protocols
    r = rng.random(n)
    f[:, 23] = np.where(r < 0.8, f[:, 23], np.where(
        r < 0.9, 1, rng.integers(0, 256, n))).astype(np.uint8)
    if valid:
        # (on a copy with a spare zero slot after the last frame: a frame
        # whose IHL was raised above has its L4 bytes run past the slot, and
        # the oracle's read of the last one must stay inside the array)
        g = np.zeros((n + 1, stride), np.uint8)
        g[:n] = f.reshape(n, stride)
        O.cksum_process(g, stride, n, 3, False)
        f.reshape(n, stride)[:] = g[:n]
    # UDP with checksum 0 (not set): stays 0
    l4 = 14 + 4 * ihl
    z = np.nonzero((f[:, 23] == 17) & (rng.random(n) < 0.2))[0]
    for i in z:
        f[i, l4[i] + 6:l4[i] + 8] = 0
    return f


# ---------------------------------------------------------------- control


def test_init_errors_match_oracle():
    from bess_amd.modules import ModuleError, StaticNAT
    bad = [
        [{"int_range": {"start": "1.2.3", "end": "1.2.3.4"},
          "ext_range": {"start": "5.6.7.8", "end": "5.6.7.8"}}],
        [{"int_range": {"start": "1.2.3.4", "end": "1.2.3.256"},
          "ext_range": {"start": "5.6.7.8", "end": "5.6.7.8"}}],
        [{"int_range": {"start": "1.2.3.5", "end": "1.2.3.4"},
          "ext_range": {"start": "5.6.7.8", "end": "5.6.7.8"}}],
        [{"int_range": {"start": "1.2.3.4", "end": "1.2.3.4"},
          "ext_range": {"start": "x", "end": "5.6.7.8"}}],
        [{"int_range": {"start": "1.2.3.4", "end": "1.2.3.4"},
          "ext_range": {"start": "5.6.7.8", "end": ""}}],
        [{"int_range": {"start": "1.2.3.4", "end": "1.2.3.4"},
          "ext_range": {"start": "5.6.7.9", "end": "5.6.7.8"}}],
        [{"int_range": {"start": "1.2.3.4", "end": "255.255.255.255"},
          "ext_range": {"start": "5.6.7.8", "end": "5.6.7.8"}}],
        [{"int_range": {"start": "1.2.3.4", "end": "1.2.3.4"},
          "ext_range": {"start": "0.0.0.0", "end": "255.255.255.255"}}],
        [{"int_range": {"start": "1.2.3.4", "end": "1.2.3.5"},
          "ext_range": {"start": "5.6.7.8", "end": "5.6.7.8"}}],
        [PAIRS[0], {"int_range": {"start": "9.9.9.9"}}],
    ]
    for pairs in bad:
        with pytest.raises(OM.OracleError) as eo:
            OM.OracleStaticNAT(pairs=pairs)
        with pytest.raises(ModuleError) as em:
            StaticNAT(pairs=pairs)
        assert em.value.code == eo.value.code == errno.EINVAL
        assert em.value.errmsg == eo.value.msg, pairs


def test_initial_arg_and_desc():
    from bess_amd.modules import StaticNAT
    m = StaticNAT(pairs=PAIRS)
    o = OM.OracleStaticNAT(pairs=PAIRS)
    got = m.get_initial_arg()
    want = o.get_initial_arg()["pairs"]
    assert len(got.pairs) == len(want)
    for g, w in zip(got.pairs, want):
        assert g.int_range.start == w["int_range"]["start"]
        assert g.int_range.end == w["int_range"]["end"]
        assert g.ext_range.start == w["ext_range"]["start"]
        assert g.ext_range.end == w["ext_range"]["end"]
    m.command("get_runtime_config")
    m.command("set_runtime_config")
    StaticNAT()  # no pairs: every packet forwarded untouched


# ----------------------------------------------------------------- oracle


def test_oracle_translation_keeps_checksums_valid():
    """IncrementalUpdateSrcIpPort (checksum_test.cc:408-457): after the
    incremental update the IPv4 and TCP/UDP checksums still verify."""
    n, stride = 4000, 256
    f = nat_frames(n, stride, seed=3, ihl_max=5)
    o = OM.OracleStaticNAT(pairs=PAIRS)
    for igate, off, want_gate in ((0, 26, 1), (1, 30, 0)):
        g = f.copy()
        out = o.process(g, stride, n, igate=igate)
        assert (out == want_gate).all()
        changed = (g[:, off:off + 4] != f[:, off:off + 4]).any(1)
        assert 0.2 < changed.mean() < 0.9
        ipg, l4g = O.cksum_process(g, stride, n, 3, True)
        tcpudp = (g[:, 23] == 6) | (g[:, 23] == 17)
        assert (ipg == 0).all() and (l4g[tcpudp] == 0).all()


def test_oracle_forward_then_reverse_restores_addresses():
    n, stride = 3000, 128
    f = nat_frames(n, stride, seed=4, ihl_max=5)
    o = OM.OracleStaticNAT(pairs=[PAIRS[2], PAIRS[3]])  # no overlaps
    g = f.copy()
    o.process(g, stride, n, igate=0)
    # move the translated source to the destination and translate back
    h = g.copy()
    h[:, 30:34] = g[:, 26:30]
    o.process(h, stride, n, igate=1)
    moved = (g[:, 26:30] != f[:, 26:30]).any(1)
    assert moved.sum() > 50
    assert (h[moved, 30:34] == f[moved, 26:30]).all()


def test_oracle_examples():
    """one translated packet, field by field"""
    o = OM.OracleStaticNAT(pairs=PAIRS)
    f = nat_frames(1, 128, seed=5, ihl_max=5)
    f[0, 23] = 17
    f[0, 26:30] = [192, 168, 1, 200]   # first pair wins over the second
    O.cksum_process(f, 128, 1, 3, False)
    g = f.copy()
    assert list(o.process(g, 128, 1, igate=0)) == [1]
    assert list(g[0, 26:30]) == [1, 2, 3, 200]
    assert list(o.process(g, 128, 1, igate=5)) == [0]  # dst not in ext ranges
    g2 = g.copy()
    g2[0, 30:34] = [1, 2, 3, 7]
    o.process(g2, 128, 1, igate=1)
    assert list(g2[0, 30:34]) == [192, 168, 1, 7]


# -------------------------------------------------------------------- GPU


@pytest.mark.gpu
@pytest.mark.parametrize("stride,ihl_max", [(64, 5), (128, 15), (2048, 15)])
@pytest.mark.parametrize("igate", [0, 1])
def test_gpu_vs_oracle(stride, ihl_max, igate):
    import torch
    from bess_amd.modules import StaticNAT
    n = 100000 if stride <= 128 else 20000
    f = nat_frames(n, stride, seed=stride + igate, valid=(igate == 0),
                   ihl_max=ihl_max)
    ref = f.copy()
    want = OM.OracleStaticNAT(pairs=PAIRS).process(ref, stride, n, igate=igate)
    m = StaticNAT(pairs=PAIRS)
    d = torch.from_numpy(f.reshape(-1)).cuda()
    og = torch.zeros(n, dtype=torch.int16, device="cuda")
    m.process_device(d, stride, n, og, igate=igate)
    assert (og.cpu().numpy().view(np.uint16) == want).all()
    got = d.cpu().numpy().reshape(n, stride)
    bad = np.nonzero((got != ref).any(1))[0]
    assert len(bad) == 0, (bad[:5], got[bad[0], :96], ref[bad[0], :96])


@pytest.mark.gpu
def test_gpu_edge_sizes():
    import torch
    from bess_amd.modules import StaticNAT
    for npairs in (0, 1, 3, 4, 5, 37):
        pairs = [pair(0x0A000000 + 0x100 * i, 0x14000000 + 0x100 * i, 256)
                 for i in range(npairs)]
        for n in (0, 1, 63, 64, 65, 1000):
            f = nat_frames(max(n, 1), 64, seed=n + npairs, ihl_max=5)[:n]
            f[:, 26] = 10
            f[:, 27] = 0
            ref = f.copy()
            want = OM.OracleStaticNAT(pairs=pairs).process(ref, 64, n)
            m = StaticNAT(pairs=pairs)
            d = torch.from_numpy(f.reshape(-1).copy()).cuda()
            og = torch.zeros(max(n, 1), dtype=torch.int16, device="cuda")
            m.process_device(d, 64, n, og)
            assert (og.cpu().numpy().view(np.uint16)[:n] == want).all()
            assert (d.cpu().numpy().reshape(n, 64) == ref).all(), (npairs, n)


@pytest.mark.gpu
def test_gpu_module_host_path_and_pipe():
    from bess_amd.modules import Pipe, StaticNAT
    m = StaticNAT(pairs=PAIRS)
    n = 30000
    f = nat_frames(n, 128, seed=9)
    ref = f.copy()
    want = OM.OracleStaticNAT(pairs=PAIRS).process(ref, 128, n, igate=1)
    g = f[:500].copy()
    assert (m.process(g, 128, 500, igate=1) == want[:500]).all()
    assert (g == ref[:500]).all()
    heads = f.ctypes.data + 128 * np.arange(n, dtype=np.uintp)
    p = Pipe(m, batch=4096, depth=3)
    assert (p.run(heads, igate=1) == want).all()
    p.close()
    assert (f == ref).all()
