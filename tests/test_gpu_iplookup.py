"""IPLookup on the GPU (DIR-16-8-8 and DIR-24-8 kernels via the module surface): gates
bit-exact against the oracle's longest-prefix match and the reference's
module tests; route tables of every depth mix, deletes revealing shorter
prefixes, default-gate changes, device slabs, the host path and the pipe."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")

from bess_amd import _lib as LB  # noqa: E402
from bess_amd import packets as P  # noqa: E402
from bess_amd.modules import IPLookup, Pipe  # noqa: E402
from oracle import oracle_more as OM  # noqa: E402


def slab(pkts, stride=2048):
    buf = np.zeros((len(pkts), stride), np.uint8)
    for i, p in enumerate(pkts):
        buf[i, :len(p)] = np.frombuffer(p, np.uint8)
    return buf


def device_gates(m, f, stride):
    d = torch.from_numpy(f.reshape(-1)).cuda()
    og = torch.zeros(len(f), dtype=torch.int16, device="cuda")
    m.process_device(d, stride, len(f), og)
    return og.cpu().numpy().view(np.uint16)


def ip(x):
    return "%d.%d.%d.%d" % ((x >> 24) & 255, (x >> 16) & 255, (x >> 8) & 255, x & 255)


def routes(n, rng, deep_frac=0.1):
    """n (prefix, len, gate): lengths 8..24 mostly, deep_frac 25..32,
    nested prefixes included"""
    out = []
    base = rng.integers(0, 1 << 32, n, dtype=np.uint64)
    for i in range(n):
        if rng.random() < deep_frac:
            plen = int(rng.integers(25, 33))
        else:
            plen = int(rng.choice([8, 12, 16, 20, 22, 23, 24]))
        if i > 0 and rng.random() < 0.3:  # nest inside an earlier route
            base[i] = base[rng.integers(0, i)]
        a = int(base[i]) & ((0xFFFFFFFF << (32 - plen)) & 0xFFFFFFFF)
        out.append((ip(a), plen, int(rng.integers(0, 64))))
    return out


def dsts_inside(rt, n, rng):
    """n destinations, each inside a uniformly picked route"""
    import ipaddress
    base = np.array([int(ipaddress.IPv4Address(p)) for p, _, _ in rt], np.uint64)
    plen = np.array([pl for _, pl, _ in rt], np.int64)
    pick = rng.integers(0, len(rt), n)
    host = rng.integers(0, np.left_shift(1, 32 - plen[pick]), dtype=np.int64)
    return base[pick] | host.astype(np.uint64)


def frames_to(dsts, stride=64):
    rng = np.random.default_rng(1)
    t = P.random_tuples(len(dsts), rng)
    t["dip"] = np.asarray(dsts, dtype=t["dip"].dtype)
    return P.build_frames(t, 60, stride)


def build(rt, max_rules=0, max_tbl8s=0):
    m = IPLookup(max_rules=max_rules, max_tbl8s=max_tbl8s)
    o = OM.OracleIPLookup(max_rules=max_rules, max_tbl8s=max_tbl8s)
    for p, plen, g in rt:
        for x in (m, o):
            try:
                x.add(prefix=p, prefix_len=plen, gate=g)
            except Exception:
                pass
    return m, o


# DIR-16-8-8 with tbl16 in LDS (the default), with tbl16 in L2 (slab and
# lane-per-packet kernels), and DIR-24-8
PATHS = [0, LB.BG_PATH_NO_LDS, LB.BG_PATH_NO_LDS | LB.BG_PATH_NO_SLAB,
         LB.BG_PATH_LPM_DIR24]


@pytest.mark.parametrize("n", [1, 5, 63, 64, 65, 2047, 64 * 1000 + 37])
def test_ragged_counts_vs_oracle(n):
    """partial last waves and workgroups (1024-thread lane-per-packet kernel,
    tbl16 in LDS; the L2 slab kernel's partial tiles)"""
    rng = np.random.default_rng(n)
    rt = routes(3000, rng, 0.05)
    m, o = build(rt, max_rules=3010, max_tbl8s=4096)
    f = frames_to(np.concatenate([dsts_inside(rt, n - n // 2, rng),
                                  rng.integers(0, 1 << 32, n // 2, dtype=np.uint64)]))
    want = o.process(f, 64, n)
    for flags in (0, LB.BG_PATH_NO_LDS):
        with LB.kernel_paths(flags):
            assert (device_gates(m, f, 64) == want).all(), flags


@pytest.mark.parametrize("flags", PATHS)
@pytest.mark.parametrize("nroutes,deep", [(1, 0.0), (100, 0.1), (5000, 0.05),
                                          (50000, 0.002), (150000, 0.0)])
def test_random_routes_vs_oracle(nroutes, deep, flags):
    rng = np.random.default_rng(nroutes)
    rt = routes(nroutes, rng, deep)
    m, o = build(rt, max_rules=nroutes + 10, max_tbl8s=4096)
    # destinations: half inside some route, half random
    rnd = rng.integers(0, 1 << 32, 40000, dtype=np.uint64)
    inside = dsts_inside(rt, 40000, rng)
    f = frames_to(np.concatenate([inside, rnd]))
    want = o.process(f, 64, len(f))
    with LB.kernel_paths(flags):
        assert (device_gates(m, f, 64) == want).all()
    assert (want != 8192).mean() > 0.4


@pytest.mark.parametrize("flags", PATHS)
def test_delete_reveals_shorter_prefix_and_default_gate(flags):
    m, o = build([("10.0.0.0", 8, 1), ("10.1.0.0", 16, 2), ("10.1.1.0", 24, 3),
                  ("10.1.1.128", 25, 4), ("10.1.1.192", 26, 5), ("10.1.1.200", 32, 6)])
    dst = [0x0A0101C8, 0x0A0101C1, 0x0A010181, 0x0A010101, 0x0A010201, 0x0A020202,
           0x0B000001]
    f = frames_to(dst, stride=128)
    steps = [None, ("delete", dict(prefix="10.1.1.200", prefix_len=32)),
             ("delete", dict(prefix="10.1.1.192", prefix_len=26)),
             ("add", dict(prefix="0.0.0.0", prefix_len=0, gate=7)),
             ("delete", dict(prefix="10.1.1.128", prefix_len=25)),
             ("delete", dict(prefix="10.1.1.0", prefix_len=24)),
             ("add", dict(prefix="10.1.1.0", prefix_len=24, gate=9)),
             ("clear", dict())]
    for st in steps:
        if st:
            getattr(m, st[0])(**st[1])
            getattr(o, st[0])(**st[1])
        with LB.kernel_paths(flags):
            assert (device_gates(m, f, 128) == o.process(f, 128, len(f))).all(), st


def test_reference_module_tests(golden):
    for case in golden("iplookup_module_kat.json"):
        m = IPLookup(**case["arg"])
        for c in case["cmds"]:
            try:
                getattr(m, c[0])(**c[1])
            except Exception:
                assert len(c) > 2
        pk = [bytes.fromhex(p) for p in case["packets"]]
        f = slab(pk)
        assert list(device_gates(m, f, 2048)) == case["expect"]
        assert list(m.process(f, 2048, len(pk))) == case["expect"]


def test_pipe():
    rng = np.random.default_rng(5)
    rt = routes(2000, rng, 0.05)
    m, o = build(rt, max_rules=4000, max_tbl8s=1024)
    f = frames_to(rng.integers(0, 1 << 32, 30000, dtype=np.uint64))
    want = o.process(f, 64, len(f))
    heads = f.ctypes.data + 64 * np.arange(len(f), dtype=np.uintp)
    p = Pipe(m, batch=4096, depth=3)
    assert (p.run(heads) == want).all()
    p.close()
