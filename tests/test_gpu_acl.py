"""ACL on the GPU (acl kernel via the module surface): output gates
bit-exact against the oracle (acl.cc restated) and the reference's module
tests, for empty / small / large ordered rule lists, drop rules, port
wildcards and every IHL, on device slabs, the host path and the pipe."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")

from bess_amd import _lib as LB  # noqa: E402
from bess_amd import packets as P  # noqa: E402
from bess_amd.modules import ACL, Pipe  # noqa: E402
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


def random_rules(n, rng, tuples):
    rules = []
    for i in range(n):
        t = tuples[rng.integers(len(tuples))]
        r = {}
        if rng.random() < 0.8:
            plen = rng.integers(0, 33) if rng.random() < 0.05 else rng.integers(16, 33)
            r["src_ip"] = "%s/%d" % (ip(int(t[0])), plen)
        if rng.random() < 0.6:
            r["dst_ip"] = "%s/%d" % (ip(int(t[1])), rng.integers(8, 33))
        if rng.random() < 0.3:
            r["src_port"] = int(t[2])
        if rng.random() < 0.3:
            r["dst_port"] = int(t[3]) if rng.random() < 0.9 else 70000 + int(t[3])
        r["drop"] = bool(rng.random() < 0.3)
        if not r.get("src_ip") and not r.get("dst_ip") and rng.random() < 0.9:
            r["src_ip"] = "%s/32" % ip(int(t[0]))
        rules.append(r)
    return rules


def workload(nrules, npkts, seed, stride=64):
    rng = np.random.default_rng(seed)
    t = P.random_tuples(max(nrules, 1), rng)
    tuples = list(zip(t["sip"], t["dip"], t["sport"], t["dport"]))
    rules = random_rules(nrules, rng, tuples)
    pk = P.random_tuples(npkts, rng)
    hit = rng.random(npkts) < 0.7
    idx = rng.integers(0, max(nrules, 1), npkts)
    for fld in pk:
        pk[fld][hit] = t[fld][idx[hit]]
    return rules, P.build_frames(pk, 60, stride)


# the default choice (the decision trees while their image fits), the rule
# scan from LDS, the scan with scalar rule loads, bit vectors forced, and
# the LDS forbidden (the scan with scalar loads)
PATHS = [0, LB.BG_PATH_ACL_LDS, LB.BG_PATH_ACL_SCAN, LB.BG_PATH_ACL_BV,
         LB.BG_PATH_NO_LDS]


def no_catch_all(rules):
    """the list without rules that match nearly everything (no address
    prefix): every tree class is populated and no scan ends early"""
    return [r for r in rules if r.get("src_ip") or r.get("dst_ip")]


@pytest.mark.parametrize("nrules", [100, 1000, 3000, 8000])
def test_trees_without_catch_all_vs_oracle(nrules):
    rules, f = workload(nrules, 60000, seed=500 + nrules)
    rules = no_catch_all(rules)
    m = ACL(rules=rules)
    o = OM.OracleACL(rules=rules)
    want = o.process(f, 64, len(f))
    assert (want == 0).any() and (want == 8192).any()
    for flags in (0, LB.BG_PATH_ACL_LDS):
        with LB.kernel_paths(flags):
            assert (device_gates(m, f, 64) == want).all()
    with LB.kernel_paths(LB.BG_PATH_NO_SLAB):  # lane-per-packet kernel
        assert (device_gates(m, f, 64) == want).all()


@pytest.mark.parametrize("flags", PATHS)
@pytest.mark.parametrize("nrules", [0, 1, 10, 31, 32, 33, 300, 3000])
def test_random_rules_vs_oracle(nrules, flags):
    rules, f = workload(nrules, 50000, seed=nrules)
    m = ACL(rules=rules)
    o = OM.OracleACL(rules=rules)
    want = o.process(f, 64, len(f))
    with LB.kernel_paths(flags):
        assert (device_gates(m, f, 64) == want).all()
    if nrules >= 10:
        assert (want == 0).any() and (want == 8192).any()


def test_rule_lists_past_the_lds_bit_vector_limit():
    """40 K rules: neither the rule list nor the address interval starts
    fit the LDS; the scan with scalar rule loads serves them -- same gates"""
    rules, f = workload(40000, 20000, seed=41)
    m = ACL(rules=rules)
    o = OM.OracleACL(rules=rules)
    want = o.process(f, 64, len(f))
    for flags in PATHS:
        with LB.kernel_paths(flags):
            assert (device_gates(m, f, 64) == want).all()


def test_wide_rules_and_many_groups():
    """2500 rules (79 rule words, summary groups of 3 words) where most
    packets match several rules and the first match lies deep in the list:
    summary bits without a single backing rule, later groups"""
    rng = np.random.default_rng(17)
    rules = []
    for i in range(2500):
        r = {"drop": bool(i % 3 == 0)}
        if i < 2400:  # narrow decoys: each dimension matches, not together
            r["src_ip"] = "10.%d.0.0/16" % (i % 50)
            r["dst_ip"] = "20.%d.0.0/16" % ((i + 7) % 50)
            r["dst_port"] = 80 + (i % 5)
        else:
            r["src_ip"] = "10.0.0.0/8"
            r["dst_port"] = 80 + (i % 7)
        rules.append(r)
    t = P.random_tuples(30000, rng)
    t["sip"][:] = (10 << 24) | rng.integers(0, 1 << 24, 30000)
    t["dip"][:] = (20 << 24) | rng.integers(0, 1 << 24, 30000)
    t["dport"][:] = 80 + rng.integers(0, 8, 30000)
    f = P.build_frames(t, 60, 64)
    m = ACL(rules=rules)
    o = OM.OracleACL(rules=rules)
    want = o.process(f, 64, len(f))
    assert (want == 0).any() and (want == 8192).any()
    for flags in PATHS:
        with LB.kernel_paths(flags):
            assert (device_gates(m, f, 64) == want).all()


@pytest.mark.parametrize("flags", PATHS)
def test_ihl_and_stride(flags):
    rules, f = workload(200, 20000, seed=7, stride=128)
    rng = np.random.default_rng(8)
    f[:, 14] = 0x40 | rng.integers(0, 16, len(f), dtype=np.uint8)
    m = ACL(rules=rules)
    o = OM.OracleACL(rules=rules)
    with LB.kernel_paths(flags):
        assert (device_gates(m, f, 128) == o.process(f, 128, len(f))).all()


def test_reference_module_tests(golden):
    for case in golden("acl_module_kat.json"):
        m = ACL(**case["arg"])
        pk = [bytes.fromhex(p) for p in case["packets"]]
        f = slab(pk)
        assert list(device_gates(m, f, 2048)) == case["expect"], case["name"]
        assert list(m.process(f, 2048, len(pk))) == case["expect"], case["name"]


def test_add_clear_and_pipe():
    rules, f = workload(100, 30000, seed=3)
    m = ACL(rules=rules[:50])
    o = OM.OracleACL(rules=rules[:50])
    m.add(rules=rules[50:])
    o.add(rules=rules[50:])
    want = o.process(f, 64, len(f))
    heads = f.ctypes.data + 64 * np.arange(len(f), dtype=np.uintp)
    p = Pipe(m, batch=4096, depth=3)
    assert (p.run(heads[:20000]) == want[:20000]).all()
    p.close()
    m.clear()
    o.clear()
    assert (device_gates(m, f, 64) == 8192).all()


def test_concurrent_workers_on_different_input_gates():
    """8 workers drive ONE ACL module at once, workers 0, 2, ... on input
    gate 0 and 1, 3, ... on input gate 1 (ctx->current_igate per call,
    core/module.h:59-75; acl.cc:70 emits a forwarded packet on it): every
    worker's gates equal the oracle's for its own input gate -- the gate
    travels with each call (bg_ctx), it is never module state. Then one
    pipe whose submits alternate input gates: each slot keeps one gate."""
    import threading
    rules, f = workload(300, 8192, seed=88)
    m = ACL(rules=rules)
    o = OM.OracleACL(rules=rules)
    want = {g: o.process(f, 64, len(f), igate=g) for g in (0, 1)}
    assert (want[0] != want[1]).any()
    heads = f.ctypes.data + 64 * np.arange(len(f), dtype=np.uintp)
    got, errs = {}, []

    def worker(w):
        try:
            outs = [m.run(heads, burst=32, igate=w % 2) for _ in range(6)]
            got[w] = outs
        except Exception as e:  # reported below
            errs.append(e)
    ths = [threading.Thread(target=worker, args=(w,)) for w in range(8)]
    for t in ths:
        t.start()
    for t in ths:
        t.join()
    assert not errs, errs
    for w in range(8):
        for g in got[w]:
            assert (g == want[w % 2]).all(), w
    # one worker's pipe fed batches from both input gates in turn
    p = Pipe(m, batch=4096, depth=3)
    for i in range(0, len(f), 32):
        p.submit(heads[i:i + 32], cookies=np.arange(i, i + 32, dtype=np.uintp),
                 igate=(i // 32) % 2)
    ck, g = p.drain()
    p.close()
    exp = np.where((ck // 32) % 2 == 1, want[1][ck], want[0][ck])
    assert len(ck) == len(f) and (ck == np.arange(len(f))).all()
    assert (g == exp).all()
