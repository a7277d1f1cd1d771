"""Module datapath on the GPU through the BESS module surface (protobuf
configured, ProcessBatch over head pointers / device slabs), bit-exact
against the oracle and the reference's module tests."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")

from bess_amd import packets as P  # noqa: E402
from bess_amd.modules import (ExactMatch, IPChecksum, L4Checksum,  # noqa: E402
                              ModuleError, WildcardMatch)
from oracle import oracle as O  # noqa: E402


def b(h):
    return bytes.fromhex(h)


def fd_from_json(x):
    if isinstance(x, dict):
        return {k: (b(v) if k == "value_bin" else fd_from_json(v))
                for k, v in x.items()}
    if isinstance(x, list):
        return [fd_from_json(v) for v in x]
    return x


def slab(pkts, stride=2048):
    buf = np.zeros((len(pkts), stride), np.uint8)
    for i, p in enumerate(pkts):
        buf[i, :len(p)] = np.frombuffer(p, np.uint8)
    return buf


@pytest.mark.parametrize("cls,kat", [(ExactMatch, "em_module_kat.json"),
                                     (WildcardMatch, "wm_module_kat.json")])
def test_module_kat(golden, cls, kat):
    dev = torch.device("cuda:0")
    for case in golden(kat):
        m = cls(**fd_from_json(case["arg"]))
        for cmd, arg in case["cmds"]:
            getattr(m, cmd)(**fd_from_json(arg))
        pk = [b(p) for p in case["packets"]]
        frames = slab(pk)
        assert list(m.process(frames, 2048, len(pk))) == case["expect"]
        d = torch.from_numpy(frames.reshape(-1)).to(dev)
        og = torch.zeros(len(pk), dtype=torch.int16, device=dev)
        m.process_device(d, 2048, len(pk), og)
        assert list(og.cpu().numpy().view(np.uint16)) == case["expect"]


def test_ip_checksum_module_kat(golden):
    k = golden("ip_checksum_module_kat.json")
    m = IPChecksum()
    frames = slab([b(c["in"]) for c in k["cases"]])
    og = m.process(frames, 2048, len(k["cases"]))
    for i, c in enumerate(k["cases"]):
        out = b(c["out"])
        assert frames[i, :len(out)].tobytes() == out, c["name"]
        assert og[i] == c["gate"]


@pytest.mark.parametrize("verify", [False, True])
def test_l4_checksum_module_vs_oracle(verify):
    frames = P.cksum_workload(2048, frame_len=590)
    if verify:  # half the frames carry correct checksums
        O.cksum_process(frames[::2], 2048, 1024, 2, False)
    ref = frames.copy()
    _, l4w = O.cksum_process(ref, 2048, 2048, 2, verify)
    og = L4Checksum(verify=verify).process(frames, 2048, 2048)
    assert (frames == ref).all() and (og == l4w).all()
    if not verify:
        assert (og == 0xFFFF).any()  # TCP frames are never emitted (P8)


def test_em_module_random_traffic_vs_oracle():
    rng = np.random.default_rng(3)
    fields = [{"offset": 23, "num_bytes": 1}, {"offset": 26, "num_bytes": 4},
              {"offset": 30, "num_bytes": 4}, {"offset": 34, "num_bytes": 2},
              {"offset": 36, "num_bytes": 2}]
    masks = [{"value_int": 0xFF}, {"value_int": 0xFFFFFF00},
             {"value_bin": b"\xff\xff\xff\xff"}, {"value_int": 0xFFFF},
             {"value_int": 0x0FFF}]
    m = ExactMatch(fields=fields, masks=masks)
    om = O.OracleExactMatch(fields=fields, masks=masks)
    keys, gates, frames = P.em_workload(3000, 50000, seed=5)
    cut = [(0, 1), (1, 5), (5, 9), (9, 11), (11, 13)]
    for k, g in zip(keys, gates):
        kb = k.tobytes()
        vals = [{"value_bin": kb[a:c]} for a, c in cut]
        # rule values: the masked bytes (value_bin = key-order bytes)
        # offset-field value_int masks are taken big-endian (P1)
        mk = [bytes([0xFF]), b"\xff\xff\xff\x00", b"\xff\xff\xff\xff",
              b"\xff\xff", b"\x0f\xff"]
        vals = [{"value_bin": bytes(x & y for x, y in zip(v["value_bin"], mm))}
                for v, mm in zip(vals, mk)]
        m.add(fields=vals, gate=int(g))
        om.add(fields=vals, gate=int(g))
    m.set_default_gate(gate=77)
    om.set_default_gate(77)
    got = m.process(frames, 64, len(frames))
    want = om.process(frames, 64, len(frames))
    assert (got == want).all()
    assert (want != 77).mean() > 0.2


def test_attr_fields_host_path_needs_metadata():
    """the synchronous host path of a module with attr_name fields: the
    attribute offsets must be bound (ENOTSUP before), and each packet's
    metadata area passed (bg_module_process_meta; EINVAL without)"""
    m = ExactMatch(fields=[{"attr_name": "foo", "num_bytes": 2}])
    m.add(fields=[{"value_bin": b"\x01\x02"}], gate=1)
    with pytest.raises(ModuleError) as e:
        m.process(np.zeros((2, 64), np.uint8), 64, 2)
    assert e.value.code == 95
    m.bind_meta(-1, {"foo": 6})
    with pytest.raises(ModuleError) as e:
        m.process(np.zeros((2, 64), np.uint8), 64, 2)
    assert e.value.code == 22


@pytest.mark.gpu
def test_attr_fields_host_path_vs_oracle():
    """bg_module_process_meta: frames and metadata areas in separate host
    buffers, bit-exact against the oracle's slot layout"""
    from test_attr_fields import ATTR_OFF, EM_FIELDS, EM_MASKS, META_OFF, STRIDE, em_rules, slots
    n = 5000
    f = slots(n, 51)
    o = O.OracleExactMatch(fields=EM_FIELDS, masks=EM_MASKS)
    m = ExactMatch(fields=EM_FIELDS, masks=EM_MASKS)
    for vals, g in em_rules(o, f, 400, np.random.default_rng(52)):
        o.add(fields=vals, gate=g)
        m.add(fields=vals, gate=g)
    want = o.process(f, STRIDE, n, meta_off=META_OFF, attr_offsets=ATTR_OFF)
    frames = np.ascontiguousarray(f[:, :META_OFF])
    meta = np.ascontiguousarray(f[:, META_OFF:])
    heads = frames.ctypes.data + META_OFF * np.arange(n, dtype=np.uintp)
    metas = meta.ctypes.data + (STRIDE - META_OFF) * np.arange(n, dtype=np.uintp)
    m.bind_meta(-1, ATTR_OFF)
    got = m.process_meta(heads, metas)
    assert (got == want).all() and (want != O.DROP_GATE).mean() > 0.02
