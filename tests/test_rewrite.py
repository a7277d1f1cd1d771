"""Rewrite (core/modules/rewrite.{h,cc}) against the oracle restatement
(oracle/oracle_more.c or_rewrite_*): the command checks and messages of
CommandAdd / CommandClear on the CPU; ProcessBatch on the GPU over device
slabs and host packet buffers, call after call (the round-robin turn).
The reference has no Rewrite test; the pin is the restated source."""
import numpy as np
import pytest

from bess_amd.modules import Rewrite
from bess_amd.modules import ModuleError
from oracle import oracle_more as OM


def templates(k, seed, lo=0, hi=1536):
    rng = np.random.default_rng(seed)
    return [rng.integers(0, 256, int(rng.integers(lo, hi + 1)), dtype=np.uint8).tobytes()
            for _ in range(k)]


def both_add(m, o, ts):
    err = None
    try:
        m.add(templates=ts)
    except ModuleError as e:
        err = (e.code, e.errmsg)
    oerr = None
    try:
        o.add(ts)
    except ValueError as e:
        oerr = e.args
    assert err == oerr
    return err


def test_add_checks_match_reference():
    m, o = Rewrite(), OM.OracleRewrite()
    assert both_add(m, o, templates(33, 1, hi=64)) == (22, "max 32 packet templates can be used 0 33")
    assert len(m) == 0
    assert both_add(m, o, templates(30, 2, hi=64)) is None
    assert both_add(m, o, templates(3, 3, hi=64)) == (22, "max 32 packet templates can be used 30 3")
    m.clear()
    o.clear()
    ts = templates(2, 4, hi=64) + [b"\0" * 1537]
    assert both_add(m, o, ts) == (22, "template is too big")
    assert len(m) == 0  # all or nothing
    assert both_add(m, o, [b"\1" * 1536, b""]) is None
    assert len(m) == 2


def slab(n, stride, seed):
    return np.random.default_rng(seed).integers(0, 256, (n, stride), dtype=np.uint8)


@pytest.mark.gpu
@pytest.mark.parametrize("k,lo,hi", [(1, 60, 60), (3, 0, 200), (7, 40, 1536), (32, 0, 1536)])
def test_gpu_vs_oracle(k, lo, hi):
    import torch
    ts = templates(k, 10 + k, lo, hi)
    m, o = Rewrite(templates=ts), OM.OracleRewrite(ts)
    stride = 2048
    for call, n in enumerate((100, 37, 1000, 1)):
        s = slab(n, stride, call)
        head = np.zeros(n, np.uint16)
        ln = np.zeros(n, np.uint32)
        d = torch.from_numpy(s.reshape(-1).copy()).cuda()
        dh = torch.zeros(n, dtype=torch.int16, device="cuda")
        dl = torch.zeros(n, dtype=torch.int32, device="cuda")
        m.process_device(d, stride, n, dh, dl)
        torch.cuda.synchronize()
        o.process(s, stride, n, head, ln)
        assert (dh.cpu().numpy().view(np.uint16) == head).all()
        assert (dl.cpu().numpy().view(np.uint32) == ln).all()
        assert (d.cpu().numpy().reshape(n, stride) == s).all(), call


@pytest.mark.gpu
def test_gpu_ordered_after_default_stream_work(default_stream_backlog):
    """stream NULL is the caller's legacy default stream: the output arrays
    are filled there behind a ~20 ms backlog right before the call, and the
    kernel must run after that fill (on a private non-blocking stream it
    ran first and the fill then overwrote every length)"""
    import torch
    ts = templates(3, 77, 0, 200)
    m, o = Rewrite(templates=ts), OM.OracleRewrite(ts)
    n, stride = 4096, 512
    s = slab(n, stride, 5)
    d = torch.from_numpy(s.reshape(-1).copy()).cuda()
    dh = torch.empty(n, dtype=torch.int16, device="cuda")
    dl = torch.empty(n, dtype=torch.int32, device="cuda")
    torch.cuda.synchronize()
    default_stream_backlog()
    dh.fill_(0x5A5A)
    dl.fill_(-1)
    m.process_device(d, stride, n, dh, dl)
    torch.cuda.synchronize()
    head = np.zeros(n, np.uint16)
    ln = np.zeros(n, np.uint32)
    o.process(s, stride, n, head, ln)
    assert (dl.cpu().numpy().view(np.uint32) == ln).all()
    assert (dh.cpu().numpy().view(np.uint16) == head).all()
    assert (d.cpu().numpy().reshape(n, stride) == s).all()


@pytest.mark.gpu
def test_gpu_host_packets_and_clear():
    """host buffers through the staging path; clear, then fewer and smaller
    templates (compared on each packet's data: the reference's sloppy copy
    takes up to 31 bytes past a size from its template slot, whose stale
    contents after a clear this port does not keep)"""
    ts = templates(5, 20, 0, 900)
    m, o = Rewrite(templates=ts), OM.OracleRewrite(ts)
    n, sb = 300, 2624
    for round_ in range(2):
        buf = slab(n, sb, 40 + round_)
        ref = buf.copy()
        ptrs = buf.ctypes.data + sb * np.arange(n, dtype=np.uintp)
        head = np.zeros(n, np.uint16)
        ln = np.zeros(n, np.uint32)
        m.process_host(ptrs, sb, head, ln)
        oh = np.zeros(n, np.uint16)
        ol = np.zeros(n, np.uint32)
        o.process(ref, sb, n, oh, ol)
        assert (head == oh).all() and (ln == ol).all()
        if round_ == 0:
            assert (buf == ref).all()
            m.clear()
            o.clear()
            ts2 = templates(2, 21, 0, 100)
            m.add(templates=ts2)
            o.add(ts2)
        else:
            for i in range(n):
                assert (buf[i, 128:128 + ln[i]] == ref[i, 128:128 + ln[i]]).all()


@pytest.mark.gpu
def test_gpu_template_change_waits_only_for_its_own_launches():
    """A template change while a batch launched on another stream is still
    queued (behind ~0.5 s of other work there): the next call uploads a new
    copy of the templates and returns without waiting for that stream or the
    device (round 5 synchronized the whole device here, so a Rewrite worker
    stalled behind every other pipe's persistent kernel -- ADVICE r05); the
    queued batch still reads the templates it was launched with."""
    import time
    import torch
    ts, ts2 = templates(3, 81, 0, 300), templates(2, 82, 0, 300)
    m, o = Rewrite(templates=ts), OM.OracleRewrite(ts)
    n, stride = 2000, 512
    s1, s2 = slab(n, stride, 1), slab(n, stride, 2)
    d1 = torch.from_numpy(s1.reshape(-1).copy()).cuda()
    d2 = torch.from_numpy(s2.reshape(-1).copy()).cuda()
    h1 = torch.zeros(n, dtype=torch.int16, device="cuda")
    l1 = torch.zeros(n, dtype=torch.int32, device="cuda")
    h2 = torch.zeros(n, dtype=torch.int16, device="cuda")
    l2 = torch.zeros(n, dtype=torch.int32, device="cuda")
    busy, other = torch.cuda.Stream(), torch.cuda.Stream()
    # the first call uploads the templates (synchronously, on its stream)
    w = slab(5, stride, 3)
    dw = torch.from_numpy(w.reshape(-1).copy()).cuda()
    hw = torch.zeros(5, dtype=torch.int16, device="cuda")
    lw = torch.zeros(5, dtype=torch.int32, device="cuda")
    m.process_device(dw, stride, 5, hw, lw, stream=other)
    o.process(w, stride, 5, np.zeros(5, np.uint16), np.zeros(5, np.uint32))
    torch.cuda.synchronize()
    with torch.cuda.stream(busy):
        torch.cuda._sleep(int(1e9))  # ~0.5 s of device work on `busy`
    m.process_device(d1, stride, n, h1, l1, stream=busy)  # queued behind it
    m.add(templates=ts2)
    t0 = time.perf_counter()
    m.process_device(d2, stride, n, h2, l2, stream=other)
    other.synchronize()
    dt = time.perf_counter() - t0
    still_busy = not busy.query()
    torch.cuda.synchronize()
    assert still_busy and dt < 0.25, dt
    for d, h, ln, s in ((d1, h1, l1, s1), (d2, h2, l2, s2)):
        oh = np.zeros(n, np.uint16)
        ol = np.zeros(n, np.uint32)
        o.process(s, stride, n, oh, ol)
        assert (h.cpu().numpy().view(np.uint16) == oh).all()
        assert (ln.cpu().numpy().view(np.uint32) == ol).all()
        got = d.cpu().numpy().reshape(n, stride)
        if s is s2:
            # past each packet's length inside its last 32-byte block the
            # reference copies its replica slot's stale bytes (CommandAdd
            # replicates templates with memcpy(size), the sloppy copy takes
            # whole blocks), which this port keeps zero: not packet data
            for i in range(n):
                end = 128 + ((int(ol[i]) + 31) & ~31)
                got[i, 128 + ol[i]:end] = s[i, 128 + ol[i]:end]
        bad = np.argwhere(got != s)
        assert len(bad) == 0, ("call 1" if s is s1 else "call 2", len(bad), bad[:4].tolist(),
                               oh[bad[:4, 0]].tolist(), ol[bad[:4, 0]].tolist())
        if s is s1:
            o.add(ts2)
