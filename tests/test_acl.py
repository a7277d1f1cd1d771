"""ACL (core/modules/acl.cc): the oracle against the reference's module
tests (bessctl/module_tests/acl.py, tests/golden/acl_module_kat.json),
Ipv4Prefix parsing semantics, and the module surface (no GPU needed)."""
import pytest

from bess_amd.modules import ACL, ModuleError
from oracle import oracle_more as OM
from oracle.oracle import OracleError


def slab(pkts, stride=2048):
    import numpy as np
    buf = np.zeros((len(pkts), stride), np.uint8)
    for i, p in enumerate(pkts):
        buf[i, :len(p)] = np.frombuffer(p, np.uint8)
    return buf


def test_oracle_vs_reference_module_tests(golden):
    for case in golden("acl_module_kat.json"):
        o = OM.OracleACL(**case["arg"])
        pk = [bytes.fromhex(p) for p in case["packets"]]
        assert list(o.process(slab(pk), 2048, len(pk))) == case["expect"], case["name"]


@pytest.mark.parametrize("prefix,want", [
    ("172.12.0.0/16", (0xAC0C0000, 0xFFFF0000)),
    ("0.0.0.0/0", (0, 0)),
    ("", (0, 0)),                      # wildcard
    ("1.2.3.4", (0, 0)),               # no '/': wildcard (ip.cc:70-73)
    ("300.1.1.1/8", (0, 0xFF000000)),  # bad address stays 0, mask applies
    ("1.2.3.4/40", (0x01020304, 0xFFFFFFFF)),
    ("1.2.3.4/-1", (0x01020304, 0xFFFFFFFF)),  # size_t(-1) >= 32
    (" 1.2.3.4/ 24", (0x01020304, 0xFFFFFF00)),
])
def test_ipv4_prefix(prefix, want):
    assert OM.ipv4_prefix(prefix) == want


def test_unparsable_length_is_an_error_not_a_crash():
    with pytest.raises(OracleError):
        OM.ipv4_prefix("1.2.3.4/")
    with pytest.raises(ModuleError) as e:
        ACL(rules=[{"src_ip": "1.2.3.4/x"}])
    assert e.value.code == 22


def test_module_commands():
    m = ACL(rules=[{"src_ip": "10.0.0.0/8"}])
    m.add(rules=[{"dst_ip": "1.2.3.0/24", "src_port": 80, "drop": True}])
    m.clear()
    assert m.desc() == ""
