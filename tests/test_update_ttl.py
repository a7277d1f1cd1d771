"""UpdateTTL (core/modules/update_ttl.cc): the oracle against the
reference's module tests (bessctl/module_tests/update_ttl.py via the golden
fixture: the decremented packet must equal a packet built with ttl - 1 and a
freshly computed checksum), plus the GPU kernel on random headers."""
import numpy as np
import pytest

from bess_amd import packets as P
from oracle import oracle_more as OM


def slab(pkts, stride=2048):
    buf = np.zeros((len(pkts), stride), np.uint8)
    for i, p in enumerate(pkts):
        buf[i, :len(p)] = np.frombuffer(p, np.uint8)
    return buf


def test_oracle_vs_reference_module_tests(golden):
    for c in golden("update_ttl_module_kat.json"):
        f = slab([bytes.fromhex(c["in"])])
        g = OM.update_ttl_process(f, 2048, 1)
        out = bytes.fromhex(c["out"])
        assert f[0, :len(out)].tobytes() == out, c["name"]
        assert g[0] == c["gate"], c["name"]


def random_headers(n, stride, seed):
    rng = np.random.default_rng(seed)
    f = P.cksum_workload(n, frame_len=min(stride, 1496) - 4 if stride > 64 else 60,
                         stride=stride, seed=seed)
    f[:, 22] = rng.integers(0, 256, n, dtype=np.uint8)        # ttl
    f[:, 24:26] = rng.integers(0, 256, (n, 2), dtype=np.uint8)  # checksum
    f[:5, 22] = [0, 1, 2, 255, 3]
    f[:5, 24:26] = [[0, 0], [0xFF, 0xFF], [0xFF, 0xFE], [0, 1], [0xFE, 0xFF]]
    return f


@pytest.mark.gpu
@pytest.mark.parametrize("stride", [64, 2048])
def test_gpu_vs_oracle(stride):
    import torch
    from bess_amd.modules import UpdateTTL
    n = 200000 if stride == 64 else 20000
    f = random_headers(n, stride, seed=stride)
    ref = f.copy()
    want = OM.update_ttl_process(ref, stride, n)
    d = torch.from_numpy(f.reshape(-1)).cuda()
    og = torch.zeros(n, dtype=torch.int16, device="cuda")
    UpdateTTL().process_device(d, stride, n, og)
    assert (og.cpu().numpy().view(np.uint16) == want).all()
    assert (d.cpu().numpy().reshape(n, stride) == ref).all()


@pytest.mark.gpu
def test_gpu_module_host_path_and_pipe(golden):
    from bess_amd.modules import Pipe, UpdateTTL
    m = UpdateTTL()
    for c in golden("update_ttl_module_kat.json"):
        f = slab([bytes.fromhex(c["in"])])
        assert list(m.process(f, 2048, 1)) == [c["gate"]]
        out = bytes.fromhex(c["out"])
        assert f[0, :len(out)].tobytes() == out
    n = 30000
    f = random_headers(n, 128, seed=9)
    ref = f.copy()
    want = OM.update_ttl_process(ref, 128, n)
    heads = f.ctypes.data + 128 * np.arange(n, dtype=np.uintp)
    p = Pipe(m, batch=4096, depth=3)
    assert (p.run(heads) == want).all()
    p.close()
    assert (f == ref).all()
