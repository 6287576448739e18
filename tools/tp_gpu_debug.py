"""Debug: TP=2 on one GPU (gloo) vs TP=1 -- token streams for several prompt sets.
Launched as: python tools/tp_gpu_debug.py  (spawns the 2 TP ranks itself)"""
import json
import os
import socket
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SETS = [[list(range(5, 40)), [100, 101], [9, 9, 9]], [[100, 101]], [[9, 9, 9]],
        [[100, 101], [9, 9, 9]], [list(range(5, 40))]]
CHILD = r"""
import json, os, sys
sys.path.insert(0, os.environ["ROOT"])
from aws_k8s_ansible_provisioner_amd.engine.config import EngineConfig, SamplingParams
from aws_k8s_ansible_provisioner_amd.parallel.tp_worker import make_tp_engine
ecfg = EngineConfig(model=os.environ["MODEL"], device="cuda", max_model_len=256, max_num_seqs=8,
                    max_num_batched_tokens=64, block_size=32, num_gpu_blocks=96,
                    tensor_parallel_size=2, shard_init="full", init_std=0.15,
                    enforce_eager=True)
eng, bc = make_tp_engine(ecfg, backend="gloo", log=lambda *a: None)
if eng is not None:
    res = []
    for ps in json.loads(os.environ["SETS"]):
        outs = eng.generate(None, SamplingParams(max_tokens=8, temperature=0, ignore_eos=True),
                            prompt_ids=ps)
        res.append([o.output_ids for o in outs])
    bc.shutdown()
    print("RESULT " + json.dumps(res), flush=True)
"""


def main():
    model = sys.argv[1] if len(sys.argv) > 1 else "tiny-llama"
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    procs = []
    for r in range(2):
        env = dict(os.environ, ROOT=ROOT, MODEL=model, RANK=str(r), WORLD_SIZE="2",
                   LOCAL_RANK=str(r), MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port),
                   SETS=json.dumps(SETS))
        procs.append(subprocess.Popen([sys.executable, "-c", CHILD], env=env,
                                      stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True))
    outs = [p.communicate(timeout=300) for p in procs]
    for p, (o, e) in zip(procs, outs):
        if p.returncode:
            print(e[-3000:])
            return 1
    got = json.loads([ln for ln in outs[0][0].splitlines() if ln.startswith("RESULT")][0][7:])
    sys.path.insert(0, ROOT)
    from aws_k8s_ansible_provisioner_amd.engine.config import EngineConfig, SamplingParams
    from aws_k8s_ansible_provisioner_amd.engine.llm_engine import LLMEngine
    from aws_k8s_ansible_provisioner_amd.models.reference_forward import dense_logits

    ref = LLMEngine(EngineConfig(model=model, device="cuda", max_model_len=256, max_num_seqs=8,
                                 max_num_batched_tokens=64, block_size=32, num_gpu_blocks=96,
                                 init_std=0.15, enforce_eager=True, shard_init="full"),
                    log=lambda *a: None)
    for ps, g in zip(SETS, got):
        want = [o.output_ids for o in ref.generate(
            None, SamplingParams(max_tokens=8, temperature=0, ignore_eos=True), prompt_ids=ps)]
        for p, a, b in zip(ps, g, want):
            seq = list(p) + list(a)
            lg = dense_logits(ref.runner.model, seq).float().cpu()
            tf_tp = [int(lg[len(p) - 1 + i].argmax()) for i in range(len(a))]
            print(f"prompt len {len(p):3d}: tp2 {a}\n               tp1 {b}\n  dense argmax on tp2 stream {tf_tp}",
                  flush=True)


if __name__ == "__main__":
    sys.exit(main() or 0)
