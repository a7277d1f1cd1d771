"""Table images retired behind the launches that read them (bg_image.cc):
batches queued on a caller's stream behind ~20 ms of other work, with a rule
change (a new image; the old one retired) between them, every batch's gates
those of the rules it was launched under -- on a stream the library does not
know (an event per launch) and on one attached with bg_stream_attach (fenced
once, at retirement)."""
import ctypes as C

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")

from bess_amd import flowtable as F  # noqa: E402
from bess_amd import lib  # noqa: E402
from bess_amd import packets as P  # noqa: E402
from oracle import oracle as O  # noqa: E402


def oracle_gates(keys, gates, frames, default_gate=8192):
    L = O.lib()
    em = L.or_em_new()
    for i, (off, size) in enumerate(P.FIVE_TUPLE):
        L.or_em_add_field(em, off, size, 0, i, None, 0)
    k = np.ascontiguousarray(keys)
    g = np.ascontiguousarray(gates, dtype=np.uint16)
    if len(k):
        assert L.or_em_add_rules(em, k.ctypes.data, len(k), k.shape[1], g.ctypes.data) == 0
    want = np.zeros(len(frames), np.uint16)
    L.or_em_process(em, frames.ctypes.data, 64, len(frames), default_gate, want.ctypes.data)
    L.or_em_free(em)
    return want


@pytest.mark.parametrize("attached", [False, True])
def test_rule_changes_behind_queued_launches(default_stream_backlog, attached):
    n, rounds = 1 << 16, 4
    keys, gates, frames = P.em_workload(4000, n, seed=31, pkt_seed=32)
    t = F.EmTable(P.em_fields_5tuple())
    step = len(keys) // rounds
    d = torch.from_numpy(frames.reshape(-1)).cuda()
    s = torch.cuda.Stream()
    sp = C.c_void_p(s.cuda_stream)
    if attached:
        assert lib().bg_stream_attach(sp) == 0
    outs, wants = [], []
    with torch.cuda.stream(s):
        default_stream_backlog()  # (torch's current stream is s here)
        for r in range(rounds):
            t.add_many(keys[r * step:(r + 1) * step], gates[r * step:(r + 1) * step])
            g = torch.full((n,), -1, dtype=torch.int16, device="cuda")
            t.classify(d, 64, n, 8192, g, stream=s)  # a new image each round
            outs.append(g)
            wants.append(oracle_gates(keys[:(r + 1) * step], gates[:(r + 1) * step], frames))
        # a fresh upload that would reuse a freed image's memory
        junk = torch.full((8 << 20,), 0x5A, dtype=torch.uint8, device="cuda")
    s.synchronize()
    del junk
    for r in range(rounds):
        assert (outs[r].cpu().numpy().view(np.uint16) == wants[r]).all(), r
    if attached:
        assert lib().bg_stream_detach(sp) == 0
