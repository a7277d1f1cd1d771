"""Module control surface (CPU): protobuf in, protobuf out, through the
bg_module_* C ABI of libbessgpu.so, checked against the reference's own
selfconfig expectations and the oracle's restatement of the control plane
(errors: code AND message)."""
import random

import pytest

from bess_amd import pb
from bess_amd.modules import (ExactMatch, IPChecksum, L4Checksum, ModuleError,
                              WildcardMatch)
from oracle import oracle as O


def b(h):
    return bytes.fromhex(h)


def fd_from_json(x):
    if isinstance(x, dict):
        return {k: (b(v) if k == "value_bin" else fd_from_json(v))
                for k, v in x.items()}
    if isinstance(x, list):
        return [fd_from_json(v) for v in x]
    return x


def same_outcome(fn_mod, fn_or):
    """Both succeed, or both fail with the same errno and message."""
    try:
        r1 = fn_mod()
        e1 = None
    except ModuleError as e:
        r1, e1 = None, (e.code, e.errmsg)
    try:
        r2 = fn_or()
        e2 = None
    except O.OracleError as e:
        r2, e2 = None, (e.code, e.msg)
    assert e1 == e2, (e1, e2)
    return r1, r2


# ----------------------------------------------------------------- proto
def test_proto_roundtrip_through_cpp():
    """Python-serialized rules -> C++ codec -> C++-serialized config ->
    Python parse."""
    em = ExactMatch(fields=[{"offset": 26, "num_bytes": 4},
                            {"offset": 30, "num_bytes": 4}])
    em.add(fields=[{"value_bin": b"\x01\x02\x03\x04"},
                   {"value_int": 0x05060708}], gate=7)
    cfg = pb.protobuf_to_dict(em.get_runtime_config())
    assert cfg == {"default_gate": 8192, "rules": [
        {"gate": 7, "fields": [{"value_bin": b"\x01\x02\x03\x04"},
                               {"value_bin": b"\x08\x07\x06\x05"}]}]}
    assert em.desc() == "2 fields, 1 rules"
    em.set_runtime_config(**cfg)
    assert pb.protobuf_to_dict(em.get_runtime_config()) == cfg


# ------------------------------------------------------------ ExactMatch
def test_em_selfconfig_kat(golden):
    c = golden("em_selfconfig_kat.json")
    em = ExactMatch(**fd_from_json(c["iconf"]))
    for cmd, arg in c["cmds"]:
        getattr(em, cmd)(**fd_from_json(arg))
    assert pb.protobuf_to_dict(em.get_initial_arg()) == \
        fd_from_json(c["expect_initial_arg"])
    assert pb.protobuf_to_dict(em.get_runtime_config()) == \
        fd_from_json(c["expect_runtime_config"])


@pytest.mark.parametrize("arg", [
    {"fields": [{"offset": 0, "num_bytes": 9}]},
    {"fields": [{"offset": 0, "num_bytes": 0}]},
    {"fields": [{"offset": 1025, "num_bytes": 1}]},
    {"fields": [{"offset": 0xFFFFFFFF, "num_bytes": 1}]},
    {"fields": [{"num_bytes": 1}]},
    {"fields": [{"offset": 0, "num_bytes": 1}], "masks": [{"value_int": 0x100}]},
    {"fields": [{"offset": 0, "num_bytes": 2}], "masks": [{"value_bin": b"\x00\x00"}]},
    {"fields": [{"offset": 0, "num_bytes": 2}, {"offset": 2, "num_bytes": 2}],
     "masks": [{"value_int": 1}]},
    {"fields": [{"offset": i, "num_bytes": 1} for i in range(9)]},
    {"fields": [{"attr_name": "a", "num_bytes": 2}, {"attr_name": "a", "num_bytes": 2}]},
    {"fields": [{"offset": 3, "num_bytes": 2}], "masks": [{"value_bin": b"\xff\x00"}]},
])
def test_em_init_errors_match_reference(arg):
    same_outcome(lambda: ExactMatch(**arg), lambda: O.OracleExactMatch(**arg))


def _random_fd(rng, size):
    if rng.random() < 0.5:
        n = size if rng.random() < 0.9 else rng.choice([size - 1, size + 1])
        return {"value_bin": bytes(rng.getrandbits(8) for _ in range(max(n, 0)))}
    return {"value_int": rng.getrandbits(8 * size + (0 if rng.random() < 0.9 else 8))}


def test_em_random_commands_vs_oracle():
    rng = random.Random(42)
    fields = [{"offset": 23, "num_bytes": 1}, {"offset": 26, "num_bytes": 4},
              {"offset": 36, "num_bytes": 2}]
    masks = [{"value_int": 0xFF}, {"value_bin": b"\xff\xff\xff\x00"},
             {"value_int": 0xFFF0}]
    em, om = ExactMatch(fields=fields, masks=masks), \
        O.OracleExactMatch(fields=fields, masks=masks)
    assert pb.protobuf_to_dict(em.get_initial_arg()) == om.get_initial_arg()
    pool = [[_random_fd(rng, s) for s in (1, 4, 2)] for _ in range(40)]
    for step in range(1500):
        r = rng.random()
        rule = rng.choice(pool)
        if r < 0.5:
            g = rng.choice([0, 1, 63, 8191, 8192, 8193, 65536 + 3, 1 << 40])
            same_outcome(lambda: em.add(fields=rule, gate=g),
                         lambda: om.add(fields=rule, gate=g))
        elif r < 0.8:
            same_outcome(lambda: em.delete(fields=rule),
                         lambda: om.delete(fields=rule))
        elif r < 0.85:
            bad = rule[:rng.randint(0, 2)]
            same_outcome(lambda: em.add(fields=bad, gate=1),
                         lambda: om.add(fields=bad, gate=1))
            same_outcome(lambda: em.delete(fields=bad),
                         lambda: om.delete(fields=bad))
        elif r < 0.9:
            g = rng.getrandbits(17)
            em.set_default_gate(gate=g)
            om.set_default_gate(g)
        elif r < 0.92:
            em.clear()
            om.clear()
        if step % 100 == 0:
            assert pb.protobuf_to_dict(em.get_runtime_config()) == \
                _drop_defaults(om.get_runtime_config())
    cfg = pb.protobuf_to_dict(em.get_runtime_config())
    assert cfg == _drop_defaults(om.get_runtime_config())
    assert em.desc() == om.get_desc()


def _drop_defaults(d):
    """oracle dicts carry every key; protobuf_to_dict omits zero scalars."""
    if isinstance(d, dict):
        return {k: _drop_defaults(v) for k, v in d.items()
                if not (v == 0 and isinstance(v, int) and k in
                        ("gate", "priority", "default_gate")) and v != []}
    if isinstance(d, list):
        return [_drop_defaults(x) for x in d]
    return d


def test_unknown_command_and_class():
    em = ExactMatch(fields=[{"offset": 0, "num_bytes": 1}])
    with pytest.raises(ModuleError) as e:
        em.command("frobnicate")
    assert e.value.code == 95  # ENOTSUP
    assert e.value.errmsg == "'ExactMatch' does not support command 'frobnicate'"
    ip = IPChecksum(verify=True)
    with pytest.raises(ModuleError) as e:
        ip.command("get_initial_arg")
    assert e.value.code == 95
    L4Checksum()


# --------------------------------------------------------- WildcardMatch
def test_wm_selfconfig_kat(golden):
    c = golden("wm_selfconfig_kat.json")
    wm = WildcardMatch(**fd_from_json(c["iconf"]))
    for cmd, arg in c["cmds"]:
        getattr(wm, cmd)(**fd_from_json(arg))
    assert pb.protobuf_to_dict(wm.get_initial_arg()) == \
        fd_from_json(c["expect_initial_arg"])
    assert pb.protobuf_to_dict(wm.get_runtime_config()) == \
        fd_from_json(c["expect_runtime_config"])


@pytest.mark.parametrize("arg", [
    {"fields": [{"offset": 0, "num_bytes": 9}]},
    {"fields": [{"offset": 2000, "num_bytes": 1}]},
    {"fields": [{"num_bytes": 2}]},
    {"fields": [{"attr_name": "", "num_bytes": 2}]},
])
def test_wm_init_errors_match_reference(arg):
    same_outcome(lambda: WildcardMatch(**arg), lambda: O.OracleWildcardMatch(**arg))


def test_wm_random_commands_vs_oracle():
    rng = random.Random(7)
    fields = [{"offset": 26, "num_bytes": 4}, {"offset": 34, "num_bytes": 2}]
    wm, ow = WildcardMatch(fields=fields), O.OracleWildcardMatch(fields=fields)
    masks = [[{"value_bin": b"\xff\xff\xff\xff"}, {"value_bin": b"\x00\x00"}],
             [{"value_int": 0xFFFF0000}, {"value_int": 0xFFFF}],
             [{"value_bin": b"\xff\x00\x00\x00"}, {"value_bin": b"\xff\xff"}]] + \
        [[{"value_int": 1 << i}, {"value_int": 0}] for i in range(8)]
    for step in range(1500):
        m = rng.choice(masks)
        v = [{"value_int": rng.getrandbits(32) & (m[0].get("value_int", 0) or 0xFF)},
             {"value_bin": bytes(rng.getrandbits(8) & 0x0F for _ in range(2))}]
        if rng.random() < 0.2:
            v = [_random_fd(rng, 4), _random_fd(rng, 2)]
        r = rng.random()
        if r < 0.5:
            g, p = rng.choice([0, 3, 8192, 9000]), rng.randint(-5, 5)
            same_outcome(lambda: wm.add(gate=g, priority=p, values=v, masks=m),
                         lambda: ow.add(gate=g, priority=p, values=v, masks=m))
        elif r < 0.8:
            same_outcome(lambda: wm.delete(values=v, masks=m),
                         lambda: ow.delete(values=v, masks=m))
        elif r < 0.82:
            wm.clear()
            ow.clear()
        elif r < 0.85:
            same_outcome(lambda: wm.add(gate=1, values=v[:1], masks=m),
                         lambda: ow.add(gate=1, values=v[:1], masks=m))
        if step % 100 == 0:
            assert pb.protobuf_to_dict(wm.get_runtime_config()) == \
                _drop_defaults(ow.get_runtime_config())
    assert pb.protobuf_to_dict(wm.get_runtime_config()) == \
        _drop_defaults(ow.get_runtime_config())
    assert wm.desc() == ow.get_desc()
