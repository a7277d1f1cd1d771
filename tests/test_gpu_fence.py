"""Rule updates while batches are in flight (bg_image.h): a THREAD_UNSAFE
command (core/module.cc:97-101; bessd runs it with the workers paused) must
not change what batches submitted before it see. A pipe holding launched
and half-filled slots, or an async classify queued on a stream, keeps the
rules of its submission: the update flushes the pipes, builds a NEW device
image at the next launch and retires the old one behind fences. Batches
submitted before the update match the old-rules oracle, later ones the new
one -- for every rule table (ExactMatch, WildcardMatch, ACL, IPLookup,
HashLB)."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")

from bess_amd import packets as P  # noqa: E402
from bess_amd.modules import (ACL, ExactMatch, HashLB, IPLookup,  # noqa: E402
                              Pipe, WildcardMatch)
from oracle import oracle as O  # noqa: E402
from oracle import oracle_more as OM  # noqa: E402

FIELDS = [{"offset": o, "num_bytes": s} for o, s in P.FIVE_TUPLE]
CUT = [(0, 1), (1, 5), (5, 9), (9, 11), (11, 13)]


def em_rule(k, g):
    kb = k.tobytes()
    return dict(fields=[{"value_bin": kb[a:b]} for a, b in CUT], gate=int(g))


def pipe_across_update(m, frames, stride, update, batch=4096, depth=4):
    """3 full slots launched plus a partial slot pending, then `update()`,
    then the rest: -> (gates in packet order, index of the first packet
    submitted after the update)"""
    n = len(frames)
    heads = frames.ctypes.data + stride * np.arange(n, dtype=np.uintp)
    p = Pipe(m, batch=batch, depth=depth)
    split = 3 * batch + 1000
    for i in range(0, split, 32):
        j = min(i + 32, split)
        p.submit(heads[i:j], cookies=np.arange(i, j, dtype=np.uintp))
    assert p.pending() == split
    update()
    for i in range(split, n, 32):
        j = min(i + 32, n)
        p.submit(heads[i:j], cookies=np.arange(i, j, dtype=np.uintp))
    ck, g = p.drain()
    p.close()
    assert (ck == np.arange(n)).all()
    return g, split


@pytest.mark.parametrize("mode", ["ring", "launch"])
def test_exact_match_pipe_across_rule_change(mode):
    """ring: slots in flight on the module's persistent kernel keep the ring
    (and its table copy) of their submission; the next slot goes to a new
    ring with the new rules"""
    from bess_amd._lib import kernel_paths, BG_PATH_PIPE_NO_RING
    with kernel_paths(BG_PATH_PIPE_NO_RING if mode == "launch" else 0):
        _exact_match_pipe_across_rule_change(1024 if mode == "ring" else 4096)


def _exact_match_pipe_across_rule_change(batch):
    keys, gates, frames = P.em_workload(1000, 40000, seed=5)
    m = ExactMatch(fields=FIELDS)
    o_old, o_new = O.OracleExactMatch(fields=FIELDS), O.OracleExactMatch(fields=FIELDS)
    for k, g in zip(keys, gates):
        m.add(**em_rule(k, g))
        o_old.add(**em_rule(k, g))
        o_new.add(**em_rule(k, (int(g) + 7) % 64))
    want_old = o_old.process(frames, 64, len(frames))
    want_new = o_new.process(frames, 64, len(frames))
    assert (want_old != want_new).sum() > 1000

    def update():  # every rule's gate changes (overwrite, P7)
        for k, g in zip(keys, gates):
            m.add(**em_rule(k, (int(g) + 7) % 64))
    got, split = pipe_across_update(m, frames, 64, update, batch=batch,
                                    depth=8 if batch == 1024 else 4)
    assert (got[:split] == want_old[:split]).all()
    assert (got[split:] == want_new[split:]).all()


def t_oracle(keys, gates, frames):
    o = O.OracleExactMatch(fields=FIELDS)
    for k, g in zip(keys, gates):
        o.add(**em_rule(k, g))
    return o.process(frames, 64, len(frames))


def test_exact_match_async_classify_across_rule_change():
    """device-slab classify queued on a side stream (8 launches), then a
    rule change and a classify on another stream: the queued launches read
    the old image to their end, the new launch the new one"""
    from bess_amd import flowtable as F
    keys, gates, frames = P.em_workload(1 << 14, 1 << 20, seed=6)
    gates2 = ((gates.astype(np.int64) + 1) % 64).astype(gates.dtype)
    t = F.EmTable(P.em_fields_5tuple())
    t.add_many(keys, gates)
    d = torch.from_numpy(frames.reshape(-1)).cuda()
    s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()
    outs = [torch.zeros(len(frames), dtype=torch.int16, device="cuda") for _ in range(8)]
    t.classify(d, 64, len(frames), 8192, outs[0])  # the first image
    torch.cuda.synchronize()
    for o in outs:
        t.classify(d, 64, len(frames), 8192, o, stream=s1)
    t.add_many(keys, gates2)  # a new image at the next launch
    new = torch.zeros(len(frames), dtype=torch.int16, device="cuda")
    t.classify(d, 64, len(frames), 8192, new, stream=s2)
    torch.cuda.synchronize()
    want_old = t_oracle(keys, gates, frames)
    want_new = t_oracle(keys, gates2, frames)
    assert (want_old != want_new).any()
    for o in outs:
        assert (o.cpu().numpy().view(np.uint16) == want_old).all()
    assert (new.cpu().numpy().view(np.uint16) == want_new).all()


def test_wildcard_match_pipe_across_rule_change():
    rk, rm, prio, wg, wf, _ = P.wm_workload(3000, 30000, stride=64, sizes=((60, 1),))
    m = WildcardMatch(fields=FIELDS)
    o_old = O.OracleWildcardMatch(fields=FIELDS)
    o_new = O.OracleWildcardMatch(fields=FIELDS)

    def rule(k, mk, p, g):
        kb, mb = k.tobytes(), mk.tobytes()
        return dict(gate=int(g), priority=int(p),
                    values=[{"value_bin": kb[a:b]} for a, b in CUT],
                    masks=[{"value_bin": mb[a:b]} for a, b in CUT])
    for k, mk, p, g in zip(rk, rm, prio, wg):
        m.add(**rule(k, mk, p, g))
        o_old.add(**rule(k, mk, p, g))
        o_new.add(**rule(k, mk, p, (int(g) + 3) % 64))
    want_old = o_old.process(wf, 64, len(wf))
    want_new = o_new.process(wf, 64, len(wf))
    assert (want_old != want_new).sum() > 1000

    def update():
        for k, mk, p, g in zip(rk, rm, prio, wg):
            m.add(**rule(k, mk, p, (int(g) + 3) % 64))
    got, split = pipe_across_update(m, wf, 64, update)
    assert (got[:split] == want_old[:split]).all()
    assert (got[split:] == want_new[split:]).all()


def test_acl_iplookup_hashlb_pipes_across_updates():
    rng = np.random.default_rng(12)
    t = P.random_tuples(30000, rng)
    frames = P.build_frames(t, 60, 64)
    # ACL: a drop rule for a third of the sources arrives mid-stream
    base = [{"src_ip": "0.0.0.0/0", "drop": False}]
    extra = [{"src_ip": "%d.0.0.0/8" % a, "drop": True} for a in range(0, 256, 3)]
    m = ACL(rules=base)
    want_old = OM.OracleACL(rules=base).process(frames, 64, len(frames))
    want_new = OM.OracleACL(rules=extra + base).process(frames, 64, len(frames))
    got, split = pipe_across_update(m, frames, 64,
                                    lambda: (m.clear(), m.add(rules=extra + base)))
    assert (got[:split] == want_old[:split]).all()
    assert (got[split:] == want_new[split:]).all()
    assert (want_old != want_new).any()
    # IPLookup: a /1 route appears
    m = IPLookup()
    o = OM.OracleIPLookup()
    m.add(prefix="0.0.0.0", prefix_len=1, gate=1)
    o.add(prefix="0.0.0.0", prefix_len=1, gate=1)
    want_old = o.process(frames, 64, len(frames))
    o.add(prefix="128.0.0.0", prefix_len=1, gate=2)
    want_new = o.process(frames, 64, len(frames))
    got, split = pipe_across_update(
        m, frames, 64, lambda: m.add(prefix="128.0.0.0", prefix_len=1, gate=2))
    assert (got[:split] == want_old[:split]).all()
    assert (got[split:] == want_new[split:]).all()
    # HashLB: the gate table changes
    m = HashLB(gates=[0, 1, 2, 3], mode="l4")
    want_old = OM.OracleHashLB(gates=[0, 1, 2, 3], mode="l4").process(frames, 64, len(frames))
    want_new = OM.OracleHashLB(gates=[4, 5, 6], mode="l4").process(frames, 64, len(frames))
    got, split = pipe_across_update(m, frames, 64, lambda: m.set_gates(gates=[4, 5, 6]))
    assert (got[:split] == want_old[:split]).all()
    assert (got[split:] == want_new[split:]).all()
