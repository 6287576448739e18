"""Timing of the IPC all-to-all / all-gather siblings of K13 (csrc/kernels/custom_allreduce.hip)
across `world` processes sharing one MI355X (the single-GPU rehearsal topology: each rank's
grid is car_grid(world) blocks).  Prints one line per (op, message bytes per rank): the
kernel time (max over ranks, CUDA events over `iters` back-to-back launches) and the
per-rank bytes moved / time.

    python tools/car_bench.py --world 2 --iters 20
"""
import argparse
import os
import socket
import sys

import torch
import torch.distributed as dist

sys.path.insert(0, os.environ.get("AKAP_REPO_ROOT")
                or os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def _port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, iters, sizes, q):
    from aws_k8s_ansible_provisioner_amd.parallel.custom_allreduce import CustomAllReduce
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank,
                            world_size=world)
    car = CustomAllReduce(group=None, device=torch.device("cuda", 0), max_bytes=1 << 20,
                          buffer_bytes=max(sizes))
    res = []
    for nbytes in sizes:
        n = nbytes // 2 // (8 * world) * (8 * world)
        send = torch.randn(n, device="cuda").to(torch.bfloat16)
        recv = torch.empty_like(send)
        rows = 256
        cols = n // rows // 8 * 8
        shard = send[:rows * cols].view(rows, cols)
        gout = torch.empty(rows, cols * world, dtype=torch.bfloat16, device="cuda")
        for op in ("all_to_all", "all_gather"):
            fn = ((lambda: car.all_to_all(send, recv)) if op == "all_to_all"
                  else (lambda: car.all_gather(shard, gout)))
            for _ in range(3):
                fn()
            torch.cuda.synchronize()
            dist.barrier()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(iters):
                fn()
            e1.record()
            torch.cuda.synchronize()
            res.append((op, n * 2, e0.elapsed_time(e1) * 1e3 / iters))
    err = car.error()
    dist.barrier()
    car.close()
    dist.destroy_process_group()
    q.put((rank, err, res))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--world", type=int, default=2)
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--sizes-mb", default="1,4,16,39")
    a = ap.parse_args()
    sizes = [int(float(s) * (1 << 20)) for s in a.sizes_mb.split(",")]
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _port()
    procs = [ctx.Process(target=_worker, args=(r, a.world, port, a.iters, sizes, q))
             for r in range(a.world)]
    for p in procs:
        p.start()
    out = {}
    for _ in range(a.world):
        r, err, res = q.get(timeout=300)
        out[r] = (err, res)
    for p in procs:
        p.join(timeout=60)
    assert all(out[r][0] == 0 for r in out), {r: out[r][0] for r in out}
    for i, (op, nb, _) in enumerate(out[0][1]):
        us = max(out[r][1][i][2] for r in out)
        print(f"{op:10s} world={a.world} {nb / 2**20:7.2f} MiB/rank  {us:8.1f} us  "
              f"{nb / us / 1e3:7.1f} GB/s/rank", flush=True)


if __name__ == "__main__":
    main()
