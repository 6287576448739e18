"""End-to-end engine on the GPU: HIP kernels + paged KV + hipGraph decode vs a dense
fp32 cache-free reference forward on the same weights (teacher-forced)."""
import pytest
import torch

from aws_k8s_ansible_provisioner_amd.engine.config import EngineConfig, SamplingParams
from aws_k8s_ansible_provisioner_amd.engine.llm_engine import LLMEngine
from aws_k8s_ansible_provisioner_amd.models.reference_forward import dense_logits

pytestmark = pytest.mark.gpu


def _engine(model, eager=False, **kw):
    cfg = dict(model=model, device="cuda", max_model_len=512, max_num_seqs=16,
               max_num_batched_tokens=128, block_size=32, num_gpu_blocks=128, init_std=0.1,
               enforce_eager=eager, cuda_graph_max_bs=16)
    cfg.update(kw)
    return LLMEngine(EngineConfig(**cfg), log=lambda *a: None)


def _check_teacher_forced(eng, prompt, out, tol=0.15):
    """Every generated token must be (near-)argmax of the dense reference logits."""
    seq = list(prompt) + list(out)
    logits = dense_logits(eng.runner.model, seq).float().cpu()
    for i, tok in enumerate(out):
        row = logits[len(prompt) - 1 + i]
        scale = row.std().item() + 1e-6
        gap = (row.max() - row[tok]).item() / scale
        assert gap <= tol, f"step {i}: token {tok} is {gap:.3f} std below the argmax"


@pytest.mark.parametrize("model", ["tiny-qwen3", "tiny-llama", "tiny-qwen3-moe"])
@pytest.mark.parametrize("eager", [False, True])
def test_engine_matches_dense_reference(model, eager):
    eng = _engine(model, eager)
    prompts = [list(range(5, 90)), [100, 101], [7, 8, 9] * 30, list(range(5, 90)),
               list(range(300, 340))]
    outs = eng.generate(None, SamplingParams(max_tokens=12, temperature=0, ignore_eos=True),
                        prompt_ids=prompts)
    assert len(outs) == len(prompts)
    for p, o in zip(prompts, outs):
        assert len(o.output_ids) == 12
        _check_teacher_forced(eng, p, o.output_ids)
    hits, queries = eng.sched.prefix_stats()
    assert hits >= 1  # the repeated prompt reused cached blocks


def test_qwen3_0_6b_shapes_one_step():
    """Real Qwen3-0.6B shapes: first generated token agrees with the dense reference."""
    eng = _engine("qwen3-0.6b", max_model_len=256, num_gpu_blocks=64, init_std=0.02)
    prompts = [list(range(1000, 1100)), list(range(50, 60))]
    outs = eng.generate(None, SamplingParams(max_tokens=3, temperature=0, ignore_eos=True),
                        prompt_ids=prompts)
    for p, o in zip(prompts, outs):
        _check_teacher_forced(eng, p, o.output_ids, tol=0.2)


def test_sampled_generation_runs_with_topk_topp():
    eng = _engine("tiny-qwen3")
    sp = SamplingParams(max_tokens=16, temperature=0.9, top_k=20, top_p=0.9, ignore_eos=True,
                        seed=7)
    a = eng.generate(None, sp, prompt_ids=[[5, 6, 7]])[0].output_ids
    b = eng.generate(None, sp, prompt_ids=[[5, 6, 7]])[0].output_ids
    assert a == b  # seeded requests are reproducible
    assert len(a) == 16


@pytest.mark.parametrize("model", ["tiny-qwen3", "tiny-llama"])
def test_engine_fp8_kv_cache(model):
    """--kv-cache-dtype fp8 end to end (fused decode + flash prefill read e4m3 bytes)."""
    eng = _engine(model, kv_cache_dtype="fp8")
    assert eng.runner.kv.dtype == torch.uint8
    prompts = [list(range(3, 80)), [17] * 33 + [5, 6, 7]]
    outs = eng.generate(None, SamplingParams(max_tokens=10, temperature=0, ignore_eos=True),
                        prompt_ids=prompts)
    for p, o in zip(prompts, outs):
        assert len(o.output_ids) == 10
        _check_teacher_forced(eng, p, o.output_ids, tol=0.6)


@pytest.mark.parametrize("model", ["tiny-qwen3", "tiny-llama"])
def test_mixed_batching_gpu(model):
    """Staggered arrivals: mixed steps run the split-KV decode kernel for the leading decode
    rows and the flash prefill kernel for the prefill rows in one eager forward; tokens are
    checked against the dense reference and equal the prefill-first policy's."""
    outs = {}
    for mixed in (True, False):
        eng = _engine(model, mixed_batching=mixed)
        sp = SamplingParams(max_tokens=8, temperature=0, ignore_eos=True)
        prompts = {"a": list(range(5, 90)), "b": [9, 8, 7] * 30, "c": list(range(300, 340))}
        eng.add_request("a", None, sp, prompt_ids=prompts["a"])
        got, saw_mixed = {}, False
        for step in range(400):
            if step == 2:
                eng.add_request("b", None, sp, prompt_ids=prompts["b"])
            if step == 4:
                eng.add_request("c", None, sp, prompt_ids=prompts["c"])
            for o in eng.step():
                if o.finished:
                    got[o.req_id] = o.output_ids
            saw_mixed |= eng.last_step_mixed
            if len(got) == 3:
                break
        assert saw_mixed == mixed
        for k, p in prompts.items():
            _check_teacher_forced(eng, p, got[k])
        outs[mixed] = got
    assert outs[True] == outs[False]


def test_qwen3_0_6b_production_decode_path():
    """Real Qwen3-0.6B shapes with max_num_seqs=64 / graphs up to 64: the GEMM tuner and the
    fused dgemm decode chain run inside the captured graphs (not only tiny models), and the
    tokens are teacher-forced against the dense reference."""
    from aws_k8s_ansible_provisioner_amd.ops import gemm_tuner

    eng = _engine("qwen3-0.6b", max_model_len=512, max_num_seqs=64, cuda_graph_max_bs=64,
                  max_num_batched_tokens=2048, num_gpu_blocks=1200, init_std=0.05)
    assert eng.runner.graphs and max(eng.runner.buckets) == 64
    assert any(gemm_tuner.fused_plan(b) is not None for b in eng.runner.buckets if b >= 16)
    prompts = [list(range(1000 + 7 * i, 1000 + 7 * i + 60 + i)) for i in range(48)]
    outs = eng.generate(None, SamplingParams(max_tokens=5, temperature=0, ignore_eos=True),
                        prompt_ids=prompts)
    assert len(outs) == 48
    for p, o in list(zip(prompts, outs))[::6]:
        _check_teacher_forced(eng, p, o.output_ids, tol=0.25)


def test_ep_decode_step_captures_in_a_hipgraph(monkeypatch):
    """Mixtral expert parallelism on 1 GPU with a simulated EP world of 1 (RCCL process group
    of size one): the fixed-capacity dispatch has no host sync, so the decode step is
    captured in hipGraphs, and the EP engine generates the tp-mode engine's tokens."""
    import os
    import socket

    import torch.distributed as dist

    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    monkeypatch.setenv("MASTER_ADDR", "127.0.0.1")
    monkeypatch.setenv("MASTER_PORT", str(port))
    created = not dist.is_initialized()
    if created:
        dist.init_process_group("nccl", rank=0, world_size=1,
                                device_id=torch.device("cuda", torch.cuda.current_device()))
    try:
        from aws_k8s_ansible_provisioner_amd.models import moe as moe_mod

        outs = {}
        for mode in ("ep", "tp"):
            monkeypatch.setenv("AKAP_MOE_MODE", mode)
            eng = _engine("tiny-mixtral")
            blk = eng.runner.model.layers[0].moe
            assert blk.mode == mode and blk.graph_safe
            assert eng.runner.graphs, f"{mode}: decode not captured"
            prompts = [list(range(5, 60)), [7, 8] * 20, list(range(200, 230))]
            res = eng.generate(None, SamplingParams(max_tokens=8, temperature=0,
                                                    ignore_eos=True), prompt_ids=prompts)
            for p, o in zip(prompts, res):
                _check_teacher_forced(eng, p, o.output_ids)
            outs[mode] = [o.output_ids for o in res]
            del eng, blk, res
        assert outs["ep"] == outs["tp"]
        # one rank: the fixed dispatch's capacity is every pair, so it can never overflow
        dev = torch.device("cuda", torch.cuda.current_device())
        assert int(moe_mod.MoEBlock.overflow_flag(dev).item()) == 0
    finally:
        if created:
            # the engines' captured hipGraphs hold RCCL work on this group's communicator:
            # free them (and let the device drain) before the communicator is destroyed
            import gc

            gc.collect()
            torch.cuda.synchronize()
            dist.destroy_process_group()


def test_async_decode_lookahead_matches_synchronous(monkeypatch):
    """Decode lookahead (step N+1 queued before step N's tokens reach the host, its input ids
    gathered on the GPU) generates exactly what the synchronous loop generates: fixed
    lengths, seeded sampling, and a stop token that ends a request while its next step is
    already in flight (that row is computed and discarded)."""
    prompts = [list(range(5, 60)), [7, 8] * 20, list(range(200, 230)), [100, 101, 102],
               list(range(400, 470))]

    def run(mode, stop_tok=None):
        monkeypatch.setenv("AKAP_ASYNC_DECODE", mode)
        eng = _engine("tiny-qwen3")
        params = [SamplingParams(max_tokens=m, temperature=0, ignore_eos=True)
                  for m in (3, 7, 12, 20)]
        params.append(SamplingParams(max_tokens=16, temperature=0.8, top_p=0.9, seed=7,
                                     ignore_eos=True))
        names = [eng.add_request(None, None, p, prompt_ids=q) for q, p in zip(prompts, params)]
        if stop_tok is not None:
            names.append(eng.add_request(None, None, SamplingParams(
                max_tokens=20, temperature=0, stop_token_ids=[stop_tok]), prompt_ids=prompts[3]))
        final = {}
        while eng.has_unfinished():
            for o in eng.step():
                if o.finished:
                    final[o.req_id] = o
        assert eng.sched.kv_usage() == 0.0
        return [final[n].output_ids for n in names], eng.lookahead_steps

    ref, n0 = run("0")
    stop_tok = ref[3][5]
    ref, _ = run("0", stop_tok)
    got, n1 = run("1", stop_tok)
    assert n0 == 0 and n1 > 10
    assert got == ref
    assert len(ref[5]) <= 6 and ref[5][-1] == stop_tok


def test_long_prompt_chunked_prefill_and_split_kv_decode():
    """Qwen3-0.6B shapes, an 8k-token prompt in 1k-token prefill chunks (each chunk's causal window reaches back
    over the cached prefix), then decode with the adaptive split-KV plan (one sequence: many
    partitions + combine), teacher-forced against the dense reference."""
    eng = _engine("qwen3-0.6b", max_model_len=16384, max_num_seqs=4, cuda_graph_max_bs=4,
                  max_num_batched_tokens=1024, num_gpu_blocks=600, init_std=0.05)
    assert eng.runner.decode_partitions(1)[0] > 1
    prompt = [int(x) for x in torch.randint(5, 1000, (8000,),
                                            generator=torch.Generator().manual_seed(0))]
    out = eng.generate(None, SamplingParams(max_tokens=6, temperature=0, ignore_eos=True),
                       prompt_ids=[prompt])[0]
    assert len(out.output_ids) == 6
    _check_teacher_forced(eng, prompt, out.output_ids, tol=0.25)


def test_pd_handoff_fills_the_v_tail_and_decodes_correctly():
    """P/D decode side on the GPU with the V tail: the prompt KV arrives as whole blocks
    (copied engine to engine in process here, in place of the RCCL transfer), activate()
    copies each prompt's partial last V group into the sequence's tail, and decoding from
    there stays teacher-forced against the dense reference."""
    pe = _engine("tiny-qwen3", kv_role="prefill")
    de = _engine("tiny-qwen3", kv_role="decode")
    assert de.runner.v_tails is not None
    prompts = [list(range(5, 50)), [100, 101, 102], list(range(200, 271)), list(range(9, 41))]
    params = SamplingParams(max_tokens=10, temperature=0, ignore_eos=True)
    for p in prompts:
        pe.add_request(None, None, params, prompt_ids=p,
                       kv_transfer_params={"do_remote_decode": True})
    done = []
    while pe.has_unfinished():
        done += [o for o in pe.step() if o.finished and o.kv_transfer_params]
    assert len(done) == len(prompts)
    bs = de.ecfg.block_size
    for o in done:
        tid = int(o.kv_transfer_params["transfer_id"])
        bp = pe.take_held(tid)
        iid, bd = de.reserve_prefilled(f"pd-{tid}", list(o.prompt_ids), int(o.output_ids[0]),
                                       params)
        assert len(bd) == len(bp)
        de.runner.kv[:, :, torch.tensor(bd)] = pe.runner.kv[:, :, torch.tensor(bp)]
        pe.finish_transfer(tid)
        de.activate(iid)
        n = len(o.prompt_ids)
        slot, cnt = de.sched.tail_slot(iid), n % 8
        assert slot >= 0
        if cnt:  # the tail holds exactly the cache's partial group
            blk, grp = bd[(n & ~7) // bs], ((n & ~7) % bs) // 8
            for vt, vc in zip(de.runner.v_tails, de.runner.v_caches):
                assert torch.equal(vt[slot, :, :cnt], vc[blk, :, grp, :, :cnt].transpose(-1, -2))
    outs = []
    while de.has_unfinished():
        outs += [o for o in de.step() if o.finished]
    assert len(outs) == len(prompts)
    for o in outs:
        assert len(o.output_ids) == 10
        _check_teacher_forced(de, o.prompt_ids, o.output_ids)


def test_inprocess_kernel_stats_window_sees_graph_replayed_kernels():
    """The in-process profiler (exporter/inprocess_profiler.py) taking a window from a side
    thread while the engine serves: the decode attention replayed from hipGraphs shows up."""
    import threading

    from aws_k8s_ansible_provisioner_amd.exporter.inprocess_profiler import InProcessKernelProfiler

    eng = _engine("tiny-qwen3")
    stop = threading.Event()

    def serve():
        while not stop.is_set():
            eng.generate(None, SamplingParams(max_tokens=32, temperature=0, ignore_eos=True),
                         prompt_ids=[[5 + i, 6, 7] for i in range(8)])

    th = threading.Thread(target=serve, daemon=True)
    th.start()
    try:
        kp = InProcessKernelProfiler(window_ms=300, interval_s=3600)
        assert kp.once(), kp.last_error
    finally:
        stop.set()
        th.join(timeout=120)
    names = " ".join(kp.windows[-1])
    assert "paged_attn_decode" in names, names[:500]
    assert "akap_kernel_profiler_up 1" in kp.text()


@pytest.mark.parametrize("model", ["tiny-qwen3", "tiny-mixtral", "tiny-qwen3-moe", "qwen3-0.6b"])
def test_prefill_on_hand_written_gemm(model, monkeypatch):
    """AKAP_PREFILL_GEMM=pgemm: every prefill projection on csrc/kernels/pgemm.hip (SwiGLU fused
    into the gate|up GEMM; Mixtral's experts on its grouped form) -- generations still match
    the dense reference."""
    from aws_k8s_ansible_provisioner_amd import ops
    from aws_k8s_ansible_provisioner_amd.models import moe

    calls = []
    real = ops.pgemm
    monkeypatch.setattr(ops, "pgemm", lambda *a, **k: calls.append(k) or real(*a, **k))
    monkeypatch.setattr(ops, "PREFILL_GEMM", "pgemm")
    monkeypatch.setattr(ops, "PGEMM_MIN_M", 16)
    monkeypatch.setattr(moe.MoEBlock, "grouped_min_t", 16)
    kw = dict(max_model_len=256, num_gpu_blocks=64, init_std=0.02) if model == "qwen3-0.6b" else {}
    eng = _engine(model, **kw)
    prompts = [list(range(5, 90)), list(range(300, 340))]
    outs = eng.generate(None, SamplingParams(max_tokens=4, temperature=0, ignore_eos=True),
                        prompt_ids=prompts)
    assert any(k.get("silu") for k in calls)
    if "mixtral" in model or "moe" in model:
        assert any(k.get("offs") is not None for k in calls)
    for p, o in zip(prompts, outs):
        _check_teacher_forced(eng, p, o.output_ids, tol=0.2)
