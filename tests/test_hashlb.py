"""HashLB (core/modules/hash_lb.cc): the oracle's CRC32C pinned by the
published CRC-32C check value, hash_range's double trick == the integer form
the kernel uses, and the module control surface (commands, errors, desc)
against the restated reference -- no GPU needed."""
import numpy as np
import pytest

from bess_amd.modules import HashLB, ModuleError
from oracle import oracle_more as OM
from oracle.oracle import OracleError


def crc32c_spec(data, crc=0):
    """bitwise reflected CRC-32C (Castagnoli 0x1EDC6F41 / reflected
    0x82F63B78), no pre/post inversion: the SSE4.2 crc32 instruction"""
    for b in data:
        crc ^= b
        for _ in range(8):
            crc = (crc >> 1) ^ (0x82F63B78 & -(crc & 1))
    return crc & 0xFFFFFFFF


def test_crc32c_spec_check_value():
    # CRC-32C check value (RFC 3720 B.4 / the CRC catalogue): "123456789"
    # with init ~0 and final inversion -> 0xE3069283
    assert crc32c_spec(b"123456789", 0xFFFFFFFF) ^ 0xFFFFFFFF == 0xE3069283


def _frames(n, seed, stride=128, ihl=None):
    rng = np.random.default_rng(seed)
    f = rng.integers(0, 256, (n, stride), dtype=np.uint8)
    if ihl is not None:
        f[:, 14] = (f[:, 14] & 0xF0) | ihl
    return f


@pytest.mark.parametrize("mode", ["l2", "l3", "l4"])
def test_oracle_crc_matches_spec(mode):
    f = _frames(300, 1, ihl=None)
    o = OM.OracleHashLB(gates=list(range(8192)), mode=mode)
    got = o.process(f, 128, len(f))
    for i in range(len(f)):
        h = f[i]
        if mode == "l2":
            s = 0
            for j in range(6):
                s ^= int(h[2 * j]) | int(h[2 * j + 1]) << 8
            crc = crc32c_spec(s.to_bytes(2, "little"))
        else:
            v0 = int.from_bytes(h[26:30].tobytes(), "little") ^ \
                int.from_bytes(h[30:34].tobytes(), "little")
            if mode == "l4":
                l4 = 14 + ((int(h[14]) & 0xF) << 2)
                v0 ^= int.from_bytes(h[l4:l4 + 2].tobytes(), "little")
                v0 ^= int.from_bytes(h[l4 + 2:l4 + 4].tobytes(), "little")
                v0 ^= int(h[23])
            crc = crc32c_spec(v0.to_bytes(4, "little"))
        assert got[i] == (crc * 8192) >> 32


def test_oracle_fields_crc_matches_spec():
    f = _frames(200, 2)
    fields = [{"offset": 23, "num_bytes": 1}, {"offset": 26, "num_bytes": 8},
              {"offset": 100, "num_bytes": 3}]
    o = OM.OracleHashLB(gates=list(range(8192)), fields=fields)
    got = o.process(f, 128, len(f))
    for i in range(len(f)):
        key = bytes(f[i, 23:24]) + bytes(f[i, 26:34]) + bytes(f[i, 100:103])
        key = key + bytes(16 - len(key))  # total_key_size 16
        assert got[i] == (crc32c_spec(key) * 8192) >> 32


def test_hash_range_is_integer_multiply_high():
    rng = np.random.default_rng(3)
    L = OM.mlib()
    for h in list(rng.integers(0, 1 << 32, 2000)) + [0, 1, 0xFFFFFFFF]:
        for r in (0, 1, 3, 7, 64, 1000, 8193, 16384):
            assert L.or_hash_range(int(h), r) == (int(h) * r) >> 32


# ---- control surface: module (libbessgpu, no device) vs oracle -------------

CASES = [
    dict(gates=[1, 2, 3]),
    dict(gates=[0, 8192], mode="l2"),
    dict(gates=[5], mode="l3"),
    dict(gates=[9], mode="bogus"),
    dict(gates=[8193]),
    dict(gates=[70000]),  # truncated to u16 (4464): valid
    dict(gates=list(range(16385))),
    dict(gates=[1], fields=[{"offset": 23, "num_bytes": 1},
                            {"offset": 26, "num_bytes": 9}]),
    dict(gates=[1], fields=[{"offset": 2000, "num_bytes": 2}]),
    dict(gates=[1], fields=[{"offset": i, "num_bytes": 1} for i in range(9)]),
    dict(gates=[1], fields=[{"attr_name": "foo", "num_bytes": 2}]),
]


def _outcome(fn):
    try:
        fn()
        return (0, "")
    except ModuleError as e:
        return (e.code, e.errmsg)
    except OracleError as e:
        return (e.code, e.msg)


@pytest.mark.parametrize("i", range(len(CASES)))
def test_init_errors_match_reference(i):
    kw = CASES[i]
    assert _outcome(lambda: HashLB(**kw)) == _outcome(lambda: OM.OracleHashLB(**kw))


def test_commands_and_desc():
    m = HashLB(gates=[1, 2])
    o = OM.OracleHashLB(gates=[1, 2])
    assert m.desc() == o.get_desc() == "0 fields"
    seq = [("set_mode", dict(mode="l3")),
           ("set_mode", dict(fields=[{"offset": 26, "num_bytes": 4},
                                     {"offset": 30, "num_bytes": 4}])),
           ("set_gates", dict(gates=[3, 4, 99999])),  # 99999 -> 34463 invalid
           ("set_mode", dict(mode="l7")),
           ("set_mode", dict(fields=[{"offset": 1, "num_bytes": 0}])),
           ("set_gates", dict(gates=list(range(20000)))),
           ("set_gates", dict(gates=[])),
           ("set_mode", dict(mode="l2"))]
    for cmd, arg in seq:
        a = _outcome(lambda: getattr(m, cmd)(**arg))
        b = _outcome(lambda: getattr(o, cmd)(**arg))
        assert a == b, (cmd, arg)
        assert m.desc() == o.get_desc()

