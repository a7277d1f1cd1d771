"""Multi-GPU plumbing for the classification path.

Packets are independent, so a node's GPUs each classify their own packet
shard with no data-path collective. The only exchange is the flow table:
when the rule set changes, rank r inserts only the rules that fall into
partition r of the ExactMatch table (every key's candidate buckets lie in
its own partition), the ranks agree on the layout with one all-reduce (MAX)
of their partition sizes, rank r builds partition r (bg_em_build_part) and
one all-gather of the partition images over RCCL (xGMI) assembles the
replicated table on every GPU (bg_em_attach). torch.distributed is the
transport only; the table bytes are produced and consumed by libbessgpu.so.
"""
import time

import numpy as np


def sharded_em_table(table, rank, world, group=None, device=None,
                     local_only=True):
    """Build + all-gather the table image. `table` holds this rank's rules:
    only partition `rank`'s (local_only, the normal case -- insert them with
    EmTable.add_many(keys, gates, part=rank, nparts=world)) or all of them.
    `device` None -> CPU tensors (gloo); otherwise a torch.device on which
    the image stays resident and is attached to `table`. Returns
    (image_tensor, stats)."""
    import torch
    import torch.distributed as dist
    t0 = time.perf_counter()
    if local_only:
        cnt = torch.tensor([table.part_count(rank, world)], dtype=torch.int64,
                           device=device)
        dist.all_reduce(cnt, op=dist.ReduceOp.MAX, group=group)
        part_bytes = table.plan_count(world, int(cnt.item()))
    else:
        part_bytes = table.plan(world)
    plan_s = time.perf_counter() - t0
    t0 = time.perf_counter()
    part = table.build_part(rank, part_bytes)
    build_s = time.perf_counter() - t0
    src = torch.from_numpy(part)
    if device is not None:
        src = src.to(device)
    full = torch.empty(part_bytes * world, dtype=torch.uint8,
                       device=src.device)
    if device is not None:
        torch.cuda.synchronize(device)
    t0 = time.perf_counter()
    dist.all_gather_into_tensor(full, src, group=group)
    if device is not None:
        torch.cuda.synchronize(device)
    ag_s = time.perf_counter() - t0
    if device is not None:
        table.attach(device.index, full)
        table._image = full  # keep the attached image alive
    return full, {"part_bytes": part_bytes, "plan_ms": plan_s * 1e3,
                  "build_ms": build_s * 1e3, "allgather_ms": ag_s * 1e3,
                  "bytes": part_bytes * world}


def local_image(table, world):
    """All partitions built in one process (reference for tests)."""
    pb = table.plan(world)
    return np.concatenate([table.build_part(p, pb) for p in range(world)])
