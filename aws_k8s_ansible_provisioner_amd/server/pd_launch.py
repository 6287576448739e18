"""Launch a disaggregated prefill/decode group inside one pod: N prefill server processes
and M decode server processes (one per GPU: prefill i on GPU i and port prefill-port + i,
decode j on GPU N + j and port decode-port + j), all ranks of one torch.distributed group.
The KV moves by the hipIpc pull (a decode process maps the prefill process's cache: any
prefill of the pod can feed any decode, so the gateway's picker pairs freely inside the
pod), or by RCCL send/recv over the group (AKAP_KV_TRANSPORT=p2p).  Default 1:1 (ports
8000 / 8001, the `pd` preset); e.g. 2:6 fills an 8-GPU node with one P/D group.

Processes are started as children before anything touches the GPU (no exec from an
initialised process); the launcher waits and exits with the first failing child's code.
"""
from __future__ import annotations

import argparse
import os
import signal
import subprocess
import sys
import time


def plan(prefill_ranks: int, decode_ranks: int, prefill_port: int = 8000,
         decode_port: int = 0) -> list[tuple[int, str, int]]:
    """[(rank, role, port)]: ranks [0, N) prefill, [N, N+M) decode (rank = local GPU)."""
    if prefill_ranks < 1 or decode_ranks < 1:
        raise ValueError("need at least one prefill and one decode rank")
    dport = decode_port or prefill_port + prefill_ranks
    out = [(i, "prefill", prefill_port + i) for i in range(prefill_ranks)]
    out += [(prefill_ranks + j, "decode", dport + j) for j in range(decode_ranks)]
    ports = [p for _, _, p in out]
    if len(set(ports)) != len(ports):
        raise ValueError(f"port collision in {out}")
    return out


def main(argv=None) -> int:
    ap = argparse.ArgumentParser("akap-pd-launch")
    ap.add_argument("--prefill-ranks", type=int, default=1)
    ap.add_argument("--decode-ranks", type=int, default=1)
    ap.add_argument("--prefill-port", type=int, default=8000)
    ap.add_argument("--decode-port", type=int, default=0,
                    help="first decode port (default prefill-port + prefill-ranks)")
    ap.add_argument("--master-port", type=int, default=29600)
    a, rest = ap.parse_known_args(argv)
    layout = plan(a.prefill_ranks, a.decode_ranks, a.prefill_port, a.decode_port)
    world = len(layout)
    procs = []
    for rank, role, port in layout:
        env = dict(os.environ, RANK=str(rank), WORLD_SIZE=str(world), LOCAL_RANK=str(rank),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(a.master_port))
        procs.append(subprocess.Popen([sys.executable, "-m", "aws_k8s_ansible_provisioner_amd.server",
                                       *rest, "--kv-role", role, "--port", str(port)], env=env))

    def stop(*_):
        for p in procs:
            if p.poll() is None:
                p.terminate()

    signal.signal(signal.SIGTERM, stop)
    signal.signal(signal.SIGINT, stop)
    while True:
        for p in procs:
            rc = p.poll()
            if rc is not None:
                stop()
                for q in procs:
                    q.wait()
                return rc
        time.sleep(1.0)


if __name__ == "__main__":
    sys.exit(main())
