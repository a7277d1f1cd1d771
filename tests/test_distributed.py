"""N>1 path on CPU: world_size 2 and 4 gloo runs of the sharded ExactMatch
table build (the only collective of the multi-GPU design): every rank
inserts only its own partition's rules, the ranks agree on the layout with
an all-reduce, build their partition and all-gather the images. The
gathered image must be byte-equal to a single-process build of the whole
rule set; the GPU test classifies packets through such a gathered image and
compares the gates with the oracle."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, n_rules, out_path, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from bess_amd import dist as D
        from bess_amd import flowtable as F
        from bess_amd import packets as P
        keys, gates, _ = P.em_workload(n_rules, 1, seed=n_rules)
        t = F.EmTable(P.em_fields_5tuple())
        t.add_many(keys, gates, part=rank, nparts=world)  # this rank's share
        held = len(t)
        full, st = D.sharded_em_table(t, rank, world)
        ref_t = F.EmTable(P.em_fields_5tuple())  # every rule, one process
        ref_t.add_many(keys, gates)
        ok = bool(np.array_equal(full.numpy(), D.local_image(ref_t, world)))
        h = torch.tensor([int(full.numpy().astype(np.uint64).sum())])
        hs = [torch.zeros_like(h) for _ in range(world)]
        dist.all_gather(hs, h)
        if rank == 0 and out_path:
            full.numpy().tofile(out_path)
        q.put((rank, ok, len(set(int(x) for x in hs)) == 1, held, st["bytes"]))
    finally:
        dist.destroy_process_group()


def run_ranks(world, n_rules, out_path=None):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_worker,
                      args=(r, world, port, n_rules, out_path, q))
          for r in range(world)]
    for p in ps:
        p.start()
    res = [q.get(timeout=300) for _ in range(world)]
    for p in ps:
        p.join(timeout=60)
        assert p.exitcode == 0
    return res


@pytest.mark.parametrize("world,n_rules", [(2, 1000), (2, 100000), (4, 20000)])
def test_sharded_table_allgather_gloo(world, n_rules):
    res = run_ranks(world, n_rules)
    assert all(ok and same for _, ok, same, _, _ in res), res
    # each rank held only its own share of the rules
    assert sum(held for _, _, _, held, _ in res) == n_rules
    assert max(held for _, _, _, held, _ in res) < n_rules


@pytest.mark.gpu
def test_gathered_image_classifies_vs_oracle(tmp_path):
    """C5 shape at world 8 on CPU ranks (gloo), then one GPU process
    attaches the gathered image and classifies 1M packets; gates must equal
    the oracle's (CuckooMap restatement holding every rule)."""
    from bess_amd import flowtable as F
    from bess_amd import packets as P
    from oracle import oracle as O
    n_rules, world = 1 << 20, 8
    img_path = str(tmp_path / "image.bin")
    res = run_ranks(world, n_rules, img_path)
    assert all(ok and same for _, ok, same, _, _ in res), res
    img = np.fromfile(img_path, np.uint8)
    keys, gates, frames = P.em_workload(n_rules, 1 << 20, seed=n_rules,
                                        pkt_seed=99)
    t = F.EmTable(P.em_fields_5tuple())
    t.add_many(keys, gates)
    assert t.plan(world) * world == img.size
    d_img = torch.from_numpy(img).cuda()
    t.attach(0, d_img)
    d_g = torch.zeros(len(frames), dtype=torch.int16, device="cuda")
    t.classify(torch.from_numpy(frames.reshape(-1)).cuda(), 64, len(frames),
               8192, d_g)
    got = d_g.cpu().numpy().view(np.uint16)
    L = O.lib()
    em = L.or_em_new()
    for i, (off, size) in enumerate(P.FIVE_TUPLE):
        L.or_em_add_field(em, off, size, 0, i, None, 0)
    k = np.ascontiguousarray(keys)
    g = np.ascontiguousarray(gates)
    assert L.or_em_add_rules(em, k.ctypes.data, len(k), k.shape[1], g.ctypes.data) == 0
    want = np.zeros(len(frames), np.uint16)
    L.or_em_process(em, frames.ctypes.data, 64, len(frames), 8192, want.ctypes.data)
    L.or_em_free(em)
    assert (got == want).all()
    assert 0.4 < (want != 8192).mean() < 0.6
