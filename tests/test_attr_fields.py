"""attr_name (metadata attribute) fields, SURVEY P15: ExactMatch reads
ptr_attr(this, attr_id, pkt) = the packet's metadata area + the attribute's
offset (exact_match.cc:230-236, core/module.h:679-684), WildcardMatch reads
buffer + mt_offset_to_databuf_offset(attr_offset) -- the same bytes
(wildcard_match.cc:177-195, packet.h:189-191). The device slot carries the
metadata area at meta_off (bg_module_bind_meta). Attribute masks are host
byte order, offset-field masks big-endian (P1).

CPU: the oracle's attr path against the same fields given as offsets, the
bind errors. GPU: module datapath vs the oracle, EM and WM, masks in both
byte orders."""
import errno

import numpy as np
import pytest

from oracle import oracle as O

STRIDE, META_OFF = 256, 128
ATTR_OFF = {"foo": 8, "bar": 21}

EM_FIELDS = [{"attr_name": "foo", "num_bytes": 2},
             {"offset": 26, "num_bytes": 4},
             {"attr_name": "bar", "num_bytes": 4}]
EM_MASKS = [{"value_int": 0xFFFF}, {"value_int": 0xFFFFFF00},
            {"value_int": 0x0FFF0FFF}]


def slots(n, seed):
    """frames in [0, 128), metadata areas in [128, 256); small alphabets so
    rules drawn from packets hit other packets too"""
    rng = np.random.default_rng(seed)
    f = rng.integers(0, 4, (n, STRIDE), dtype=np.uint8)
    return f


def src_bytes(f, i, fd, size):
    off = META_OFF + ATTR_OFF[fd["attr_name"]] if "attr_name" in fd else fd["offset"]
    return f[i, off:off + size].tobytes()


def em_rules(o, f, k, rng):
    rules = []
    for i in rng.choice(len(f), k, replace=False):
        vals = []
        for j, fd in enumerate(EM_FIELDS):
            fl = o.field(j)
            b = src_bytes(f, i, fd, fl["size"])
            m = fl["mask"].to_bytes(8, "little")[:fl["size"]]
            vals.append({"value_bin": bytes(x & y for x, y in zip(b, m))})
        rules.append((vals, int(rng.integers(0, 64))))
    return rules


def test_oracle_attr_path_reads_metadata():
    """unmasked attr fields == offset fields at meta_off + attr offset"""
    f = slots(3000, 1)
    rng = np.random.default_rng(2)
    fa = [{"attr_name": "foo", "num_bytes": 2}, {"offset": 26, "num_bytes": 4},
          {"attr_name": "bar", "num_bytes": 3}]
    fo = [{"offset": META_OFF + 8, "num_bytes": 2}, {"offset": 26, "num_bytes": 4},
          {"offset": META_OFF + 21, "num_bytes": 3}]
    a, b = O.OracleExactMatch(fields=fa), O.OracleExactMatch(fields=fo)
    for i in rng.choice(3000, 300, replace=False):
        vals = [{"value_bin": src_bytes(f, i, fd, fd["num_bytes"])} for fd in fa]
        g = int(rng.integers(0, 64))
        a.add(fields=vals, gate=g)
        b.add(fields=vals, gate=g)
    ga = a.process(f, STRIDE, 3000, meta_off=META_OFF, attr_offsets=ATTR_OFF)
    gb = b.process(f, STRIDE, 3000)
    assert (ga == gb).all() and (ga != O.DROP_GATE).mean() > 0.1
    with pytest.raises(O.OracleError):
        a.process(f, STRIDE, 10)  # no metadata layout: no datapath


def test_bind_errors():
    from bess_amd.modules import ExactMatch, IPChecksum, ModuleError, WildcardMatch
    m = ExactMatch(fields=EM_FIELDS, masks=EM_MASKS)
    with pytest.raises(ModuleError) as e:
        m.bind_meta(META_OFF, {"foo": 8})            # 'bar' unplaced
    assert e.value.code == errno.EINVAL and "attribute 1" in e.value.errmsg
    with pytest.raises(ModuleError) as e:
        m.bind_meta(-4, ATTR_OFF)
    assert e.value.code == errno.EINVAL
    with pytest.raises(ModuleError) as e:
        m.bind_meta(2040, ATTR_OFF)                   # past the 2 KB slot
    assert e.value.code == errno.EINVAL
    m.bind_meta(META_OFF, dict(ATTR_OFF, other=3))    # extra names ignored
    w = WildcardMatch(fields=[{"attr_name": "x", "num_bytes": 1}])
    w.bind_meta(0, {"x": 5})
    with pytest.raises(ModuleError) as e:
        IPChecksum().bind_meta(0, {})
    assert e.value.code == errno.ENOTSUP


@pytest.mark.gpu
def test_gpu_em_attr_fields_vs_oracle():
    import torch
    from bess_amd.modules import ExactMatch, ModuleError
    n = 50000
    f = slots(n, 3)
    o = O.OracleExactMatch(fields=EM_FIELDS, masks=EM_MASKS)
    m = ExactMatch(fields=EM_FIELDS, masks=EM_MASKS)
    for vals, g in em_rules(o, f, 2000, np.random.default_rng(4)):
        o.add(fields=vals, gate=g)
        m.add(fields=vals, gate=g)
    m.set_default_gate(gate=70)
    o.set_default_gate(70)
    want = o.process(f, STRIDE, n, meta_off=META_OFF, attr_offsets=ATTR_OFF)
    d = torch.from_numpy(f.reshape(-1)).cuda()
    og = torch.zeros(n, dtype=torch.int16, device="cuda")
    with pytest.raises(ModuleError) as e:            # not bound yet
        m.process_device(d, STRIDE, n, og)
    assert e.value.code == errno.ENOTSUP
    m.bind_meta(META_OFF, ATTR_OFF)
    m.process_device(d, STRIDE, n, og)
    got = og.cpu().numpy().view(np.uint16)
    assert (got == want).all()
    assert (want != 70).mean() > 0.02
    # offsets only (a host datapath's bind): the slab layout bound before
    # is gone, so the device-slab call is unbound again
    m.bind_meta(-1, ATTR_OFF)
    with pytest.raises(ModuleError) as e:
        m.process_device(d, STRIDE, n, og)
    assert e.value.code == errno.ENOTSUP


@pytest.mark.gpu
def test_gpu_wm_attr_fields_vs_oracle():
    import torch
    from bess_amd.modules import WildcardMatch
    fields = [{"attr_name": "foo", "num_bytes": 2}, {"offset": 30, "num_bytes": 4},
              {"attr_name": "bar", "num_bytes": 1}]
    n = 50000
    f = slots(n, 5)
    rng = np.random.default_rng(6)
    masks = [[b"\xff\xff", b"\x00\x00\x00\x00", b"\x00"],
             [b"\x00\x00", b"\xff\xff\xff\x00", b"\x03"],
             [b"\xff\x00", b"\x00\x00\x00\x00", b"\xff"]]
    o = O.OracleWildcardMatch(fields=fields)
    m = WildcardMatch(fields=fields)
    for i in rng.choice(n, 600, replace=False):
        mk = masks[int(rng.integers(0, 3))]
        vals = [bytes(x & y for x, y in zip(src_bytes(f, i, fd, fd["num_bytes"]), mb))
                for fd, mb in zip(fields, mk)]
        arg = dict(gate=int(rng.integers(0, 64)), priority=int(rng.integers(0, 5)),
                   values=[{"value_bin": v} for v in vals],
                   masks=[{"value_bin": mb} for mb in mk])
        o.add(**arg)
        m.add(**arg)
    want = o.process(f, STRIDE, n, meta_off=META_OFF, attr_offsets=ATTR_OFF)
    m.bind_meta(META_OFF, ATTR_OFF)
    d = torch.from_numpy(f.reshape(-1)).cuda()
    og = torch.zeros(n, dtype=torch.int16, device="cuda")
    m.process_device(d, STRIDE, n, og)
    got = og.cpu().numpy().view(np.uint16)
    assert (got == want).all()
    assert (want != O.DROP_GATE).mean() > 0.05
