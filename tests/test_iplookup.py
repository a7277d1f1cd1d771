"""IPLookup (core/modules/ip_lookup.cc): oracle against the reference's
module tests (bessctl/module_tests/iplookup.py, golden fixture), and the
module control surface -- errors, messages, rte_lpm capacity semantics --
against the restated reference (no GPU needed)."""
import pytest

from bess_amd.modules import IPLookup, ModuleError
from oracle import oracle_more as OM
from oracle.oracle import OracleError


def slab(pkts, stride=2048):
    import numpy as np
    buf = np.zeros((len(pkts), stride), np.uint8)
    for i, p in enumerate(pkts):
        buf[i, :len(p)] = np.frombuffer(p, np.uint8)
    return buf


def _outcome(fn):
    try:
        fn()
        return (0, "")
    except ModuleError as e:
        return (e.code, e.errmsg)
    except OracleError as e:
        return (e.code, e.msg)


def test_oracle_vs_reference_module_tests(golden):
    for case in golden("iplookup_module_kat.json"):
        o = OM.OracleIPLookup(**case["arg"])
        m = IPLookup(**case["arg"])
        for c in case["cmds"]:
            cmd, arg = c[0], c[1]
            a = _outcome(lambda: getattr(o, cmd)(**arg))
            b = _outcome(lambda: getattr(m, cmd)(**arg))
            assert a == b
            assert (a[0] != 0) == (len(c) > 2 and c[2] == "error"), (case["name"], c)
        pk = [bytes.fromhex(p) for p in case["packets"]]
        assert list(o.process(slab(pk), 2048, len(pk))) == case["expect"]


CMDS = [
    ("add", dict(prefix="", prefix_len=8, gate=1)),
    ("add", dict(prefix="1.2.3", prefix_len=8, gate=1)),
    ("add", dict(prefix="1.2.3.4", prefix_len=33, gate=1)),
    ("add", dict(prefix="10.0.0.0", prefix_len=8, gate=9000)),
    ("add", dict(prefix="10.0.0.0", prefix_len=8, gate=8192)),
    ("add", dict(prefix="10.0.0.0", prefix_len=8, gate=3)),     # update
    ("add", dict(prefix="0.0.0.0", prefix_len=0, gate=5)),      # default gate
    ("delete", dict(prefix="0.0.0.0", prefix_len=0)),
    ("delete", dict(prefix="11.0.0.0", prefix_len=8)),
    ("add", dict(prefix="10.1.1.128", prefix_len=25, gate=4)),
    ("add", dict(prefix="10.1.1.0", prefix_len=25, gate=4)),    # same block
    ("add", dict(prefix="10.1.2.0", prefix_len=26, gate=4)),    # 2nd tbl8
    ("add", dict(prefix="10.1.3.0", prefix_len=26, gate=4)),    # no tbl8 left
    ("delete", dict(prefix="10.1.2.0", prefix_len=26)),         # recycled
    ("add", dict(prefix="10.1.3.0", prefix_len=26, gate=4)),
    ("add", dict(prefix="20.0.0.0", prefix_len=8, gate=1)),
    ("add", dict(prefix="21.0.0.0", prefix_len=8, gate=1)),     # max_rules
    ("clear", dict()),
    ("add", dict(prefix="21.0.0.0", prefix_len=8, gate=1)),
]


def test_control_surface_matches_reference():
    m = IPLookup(max_rules=6, max_tbl8s=2)
    o = OM.OracleIPLookup(max_rules=6, max_tbl8s=2)
    for cmd, arg in CMDS:
        a = _outcome(lambda: getattr(m, cmd)(**arg))
        b = _outcome(lambda: getattr(o, cmd)(**arg))
        assert a == b, (cmd, arg, a, b)
    assert _outcome(lambda: o.add(prefix="1.2.3.4", prefix_len=33, gate=1)) == \
        (22, "Invalid prefix length: 33")
    assert _outcome(lambda: o.add(prefix="22.22.22.0", prefix_len=16, gate=0)) == \
        (22, "Invalid IP prefix 22.22.22.0/16 16161600 ffff0000")


def test_cpu_baseline_dir24_equals_oracle():
    """The CPU baseline times rte_lpm's DIR-24-8 lookup (restated in
    oracle_more.c, DPDK being absent); it must give the oracle's longest-
    prefix results (an independent per-depth search) on nested routes."""
    import numpy as np
    rng = np.random.default_rng(3)
    o = OM.OracleIPLookup(max_rules=5000, max_tbl8s=2000)
    for _ in range(3000):
        d = int(rng.choice([8, 12, 16, 20, 24, 25, 28, 30, 32]))
        ip = int(rng.integers(0, 1 << 32)) & ((0xFFFFFFFF << (32 - d)) & 0xFFFFFFFF)
        o.add(prefix="%d.%d.%d.%d" % tuple(ip.to_bytes(4, "big")), prefix_len=d,
              gate=int(rng.integers(0, 8000)))
    n = 20000
    frames = np.zeros((n, 64), np.uint8)
    keys = [ip for ip, _ in o.rules]
    dst = np.where(rng.random(n) < 0.7,
                   np.array(keys)[rng.integers(0, len(keys), n)] +
                   rng.integers(0, 256, n), rng.integers(0, 1 << 32, n)) & 0xFFFFFFFF
    frames[:, 30:34] = dst.astype(">u4").view(np.uint8).reshape(n, 4)
    want = o.process(frames, 64, n)
    t = o.dir24()
    got = np.zeros(n, np.uint16)
    OM.mlib().or_dir24_process(t, frames.ctypes.data, 64, n, o.default_gate,
                               got.ctypes.data)
    OM.mlib().or_dir24_free(t)
    assert (got == want).all()
    assert (want != o.default_gate).mean() > 0.3
