"""The rule-table collective through the C ABI (bg_comm_*, bg_em_allgather*,
RCCL over xGMI, no torch.distributed): a C++ host builds the sharded C5
ExactMatch image itself. On a one-GPU box the communicators have one rank:
bg_comm_init_all([0]) with the grouped in-process build, and
bg_comm_unique_id + bg_comm_init_rank(1 rank) with the per-rank build from a
table holding only its partition's rules. The image each produces must give
the oracle's gates (the world-2/4 gathers run on CPU in test_distributed)."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")

from bess_amd import flowtable as F  # noqa: E402
from bess_amd import packets as P  # noqa: E402
from oracle import oracle as O  # noqa: E402


def oracle_gates(keys, gates, frames):
    L = O.lib()
    em = L.or_em_new()
    for i, (off, size) in enumerate(P.FIVE_TUPLE):
        L.or_em_add_field(em, off, size, 0, i, None, 0)
    k = np.ascontiguousarray(keys)
    g = np.ascontiguousarray(gates, dtype=np.uint16)
    L.or_em_add_rules(em, k.ctypes.data, len(k), k.shape[1], g.ctypes.data)
    want = np.zeros(len(frames), np.uint16)
    L.or_em_process(em, frames.ctypes.data, 64, len(frames), 8192, want.ctypes.data)
    L.or_em_free(em)
    return want


@pytest.fixture(scope="module")
def workload():
    keys, gates, frames = P.em_workload(1 << 18, 1 << 20, seed=77)
    return keys, gates, frames, oracle_gates(keys, gates, frames)


def classify(t, frames):
    d = torch.from_numpy(frames.reshape(-1)).cuda()
    g = torch.zeros(len(frames), dtype=torch.int16, device="cuda")
    t.classify(d, 64, len(frames), 8192, g)
    torch.cuda.synchronize()
    return g.cpu().numpy().view(np.uint16)


def test_init_all_grouped_allgather(workload):
    keys, gates, frames, want = workload
    comms = F.Comm.init_all([0])
    assert comms[0].info() == (0, 1, 0)
    t = F.EmTable(P.em_fields_5tuple())
    t.add_many(keys, gates)
    t.allgather_all(comms)
    nbytes, _ = t.table_info()
    assert nbytes > 0
    assert (classify(t, frames) == want).all()
    # a rule change after the gather: the next launch rebuilds from the rules
    t.add_many(keys[:1000], (gates[:1000].astype(np.int64) + 1) % 64)
    g2 = gates.copy()
    g2[:1000] = (g2[:1000].astype(np.int64) + 1) % 64
    assert (classify(t, frames) == oracle_gates(keys, g2, frames)).all()
    for c in comms:
        c.close()


def test_init_rank_allgather_from_own_partition(workload):
    keys, gates, frames, want = workload
    uid = F.Comm.unique_id()
    c = F.Comm.init_rank(uid, 1, 0, 0)
    assert c.info() == (0, 1, 0)
    t = F.EmTable(P.em_fields_5tuple())
    t.add_many(keys, gates, part=0, nparts=1)  # this rank's share (all, at 1)
    t.allgather(c)
    assert (classify(t, frames) == want).all()
    c.close()
