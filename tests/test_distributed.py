"""N>1 path on CPU: world_size-2 gloo all-gather of the sharded ExactMatch
table image (the only collective of the multi-GPU design)."""
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


def _worker(rank, world, port, n_rules, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from bess_amd import dist as D
        from bess_amd import flowtable as F
        from bess_amd import packets as P
        keys, gates, _ = P.em_workload(n_rules, 1)  # same rules on every rank
        t = F.EmTable(P.em_fields_5tuple())
        t.add_many(keys, gates)
        full, st = D.sharded_em_table(t, rank, world)
        ref = D.local_image(t, world)
        ok = bool(np.array_equal(full.numpy(), ref))
        # identical on every rank
        h = torch.tensor([int(np.frombuffer(full.numpy().tobytes()[:1 << 20],
                                            np.uint8).sum())])
        hs = [torch.zeros_like(h) for _ in range(world)]
        dist.all_gather(hs, h)
        q.put((rank, ok, len(set(int(x) for x in hs)) == 1, st["bytes"]))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,n_rules", [(2, 1000), (2, 100000), (4, 20000)])
def test_sharded_table_allgather_gloo(world, n_rules):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_worker, args=(r, world, port, n_rules, q))
          for r in range(world)]
    for p in ps:
        p.start()
    res = [q.get(timeout=240) for _ in range(world)]
    for p in ps:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert all(ok and same for _, ok, same, _ in res), res
