"""Launch a disaggregated prefill/decode pair inside one pod: two server processes
(prefill on GPU 0 / :prefill-port, decode on GPU 1 / :decode-port) forming one
torch.distributed group (RCCL over xGMI) for KV-cache transfer.

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


def main(argv=None) -> int:
    ap = argparse.ArgumentParser("akap-pd-launch")
    ap.add_argument("--prefill-port", type=int, default=8000)
    ap.add_argument("--decode-port", type=int, default=8001)
    ap.add_argument("--master-port", type=int, default=29600)
    a, rest = ap.parse_known_args(argv)
    procs = []
    for rank, (role, port) in enumerate([("prefill", a.prefill_port), ("decode", a.decode_port)]):
        env = dict(os.environ, RANK=str(rank), WORLD_SIZE="2", LOCAL_RANK=str(rank),
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
