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
