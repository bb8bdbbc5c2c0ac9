"""Probe: can two ranks share one MI355X under the nccl (= RCCL) backend?  Spawns 2 processes on cuda:0, each
all-reduces a tensor and checks the sum.  Prints one JSON line.  (The 8-GPU scaling run is the driver's; this
only asks whether a 1-GPU box can execute a multi-rank RCCL group at all.)

    python benchmarks/rccl_two_ranks_one_gpu.py
"""
import json
import os
import socket
import sys

import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def _port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    try:
        dev = torch.device("cuda", 0)
        torch.cuda.set_device(dev)
        dist.init_process_group("nccl", rank=rank, world_size=world, device_id=dev)
        x = torch.full((1 << 20,), float(rank + 1), device=dev)
        dist.all_reduce(x)
        torch.cuda.synchronize()
        ok = bool((x == sum(range(1, world + 1))).all())
        dist.destroy_process_group()
        q.put((rank, ok, ""))
    except Exception as e:  # noqa: BLE001 -- report, do not hang
        q.put((rank, False, repr(e)[:300]))


def main():
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _port()
    ps = [ctx.Process(target=worker, args=(r, world, port, q)) for r in range(world)]
    for p in ps:
        p.start()
    res = [q.get(timeout=120) for _ in range(world)]
    for p in ps:
        p.join(30)
    print(json.dumps({"probe": "rccl 2 ranks on 1 GPU", "results": sorted(res)}), flush=True)
    sys.exit(0 if all(r[1] for r in res) else 3)


if __name__ == "__main__":
    main()
