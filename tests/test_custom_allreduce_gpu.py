"""Custom xGMI all-reduce kernels (K13) on one MI355X.

* in-process: W communicators in one process (one per simulated rank) wired together
  without IPC, all ranks in one grid (blockIdx.y = rank, so co-residency does not depend
  on the stream -> hardware-queue mapping) or, for W=2, on two HIP streams -- exercises
  the flag protocol, epoch parity, slice ownership and graph replay;
* multi-process: 2 processes on the same GPU exchange real hipIpc handles over gloo.
Results are checked against an fp32 sum of the inputs (PyTorch reference)."""
import socket

import pytest
import torch

from aws_k8s_ansible_provisioner_amd import ops

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _ref_sum(xs):
    acc = torch.zeros_like(xs[0], dtype=torch.float32)
    for x in xs:
        acc += x.float()
    return acc.to(torch.bfloat16)


def _explain(outs, exp, prev, r, world, n, two_shot):
    """Self-explaining failure: first bad element, its block/lane, and what it equals."""
    d = (outs[r].float() - exp.float()).abs()
    bad = (~(d <= 0.02 * world)).nonzero().flatten()
    i = int(bad[0])
    v = outs[r][i].float().item()
    n8 = n // 8
    per = (n8 + world - 1) // world if two_shot else n8
    nblk = max(1, min(128, (per + 255) // 256))
    vec = i // 8
    kind = "unwritten (NaN)" if v != v else (
        "previous epoch's sum" if prev is not None and abs(v - prev[i].float().item()) <= 0.04
        else "other")
    return (f"rank {r}: {len(bad)} bad of {n}; first elem {i} (vector {vec}, block "
            f"{(vec % (nblk * 256)) // 256}, lane {vec % 256}) = {v} vs {exp[i].item()}: {kind}")


@pytest.mark.parametrize("world", [2, 3, 4, 8])
@pytest.mark.parametrize("two_shot", [False, True])
@pytest.mark.parametrize("n", [8, 4096, 8 * 1000 + 8 * 3, 1 << 19])
def test_custom_allreduce_in_process(world, two_shot, n):
    """All simulated ranks in one grid (blockIdx.y = rank): protocol, parity, ownership.
    Outputs are poisoned with NaN before every call (an unwritten element cannot pass), and
    every other epoch the consumers pre-read the peers' staging lines with plain loads (an
    L1/L2-warm consumer: a protocol relying on a cache invalidate would read them stale)."""
    ops.load_native(required=True)
    max_elems = 1 << 20
    hs = [torch.ops.akap.car_create(0, r, world, max_elems) for r in range(world)]
    prev = None
    try:
        for h in hs:
            torch.ops.akap.car_link_local(h, hs)
        for it in range(6):  # several epochs: both parities, reused flags, warm and cold
            torch.manual_seed(100 * it + world + n)
            xs = [torch.randn(n, dtype=torch.bfloat16, device=DEV) for _ in range(world)]
            outs = [torch.full_like(x, float("nan")) for x in xs]
            torch.ops.akap.car_all_reduce_multi(hs, xs, outs, two_shot, None, it % 2 == 1)
            torch.cuda.synchronize()
            for h in hs:
                assert torch.ops.akap.car_error(h) == 0, "flag wait timed out"
            exp = _ref_sum(xs)
            for r in range(world):
                err = (outs[r].float() - exp.float()).abs().max().item()
                assert err <= 0.02 * world, f"epoch {it}: " + _explain(outs, exp, prev, r, world,
                                                                      n, two_shot)
                assert torch.equal(outs[r], outs[0]), "ranks disagree"
            prev = exp
    finally:
        torch.cuda.synchronize()
        for h in hs:
            torch.ops.akap.car_destroy(h)


def test_custom_allreduce_two_streams():
    """Two ranks as separate launches on separate HIP streams (the production launch)."""
    ops.load_native(required=True)
    world, n = 2, 40000
    hs = [torch.ops.akap.car_create(0, r, world, 1 << 16) for r in range(world)]
    try:
        for h in hs:
            torch.ops.akap.car_link_local(h, hs)
        streams = [torch.cuda.Stream() for _ in range(world)]
        for it in range(3):
            xs = [torch.randn(n, dtype=torch.bfloat16, device=DEV) for _ in range(world)]
            outs = [torch.empty_like(x) for x in xs]
            torch.cuda.synchronize()
            for r in range(world):
                with torch.cuda.stream(streams[r]):
                    torch.ops.akap.car_all_reduce(hs[r], xs[r], outs[r], False)
            torch.cuda.synchronize()
            assert all(torch.ops.akap.car_error(h) == 0 for h in hs)
            assert torch.equal(outs[0], outs[1])
            assert (outs[0].float() - _ref_sum(xs).float()).abs().max().item() <= 0.05
    finally:
        torch.cuda.synchronize()
        for h in hs:
            torch.ops.akap.car_destroy(h)


def test_custom_allreduce_graph_replay():
    """Captured once, replayed several times: the device-side epochs must advance."""
    ops.load_native(required=True)
    world, n = 4, 8192
    hs = [torch.ops.akap.car_create(0, r, world, 1 << 14) for r in range(world)]
    try:
        for h in hs:
            torch.ops.akap.car_link_local(h, hs)
        xs = [torch.randn(n, dtype=torch.bfloat16, device=DEV) for _ in range(world)]
        outs = [torch.empty_like(x) for x in xs]
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            torch.ops.akap.car_all_reduce_multi(hs, xs, outs, True)
        torch.cuda.current_stream().wait_stream(s)
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            torch.ops.akap.car_all_reduce_multi(hs, xs, outs, True)
        for it in range(4):
            for x in xs:
                x.copy_(torch.randn(n, dtype=torch.bfloat16, device=DEV))
            g.replay()
            torch.cuda.synchronize()
            assert all(torch.ops.akap.car_error(h) == 0 for h in hs)
            assert (outs[2].float() - _ref_sum(xs).float()).abs().max().item() <= 0.1
    finally:
        torch.cuda.synchronize()
        for h in hs:
            torch.ops.akap.car_destroy(h)


def test_custom_allreduce_in_place():
    ops.load_native(required=True)
    world, n = 2, 2048
    hs = [torch.ops.akap.car_create(0, r, world, 4096) for r in range(world)]
    try:
        for h in hs:
            torch.ops.akap.car_link_local(h, hs)
        xs = [torch.randn(n, dtype=torch.bfloat16, device=DEV) for _ in range(world)]
        exp = _ref_sum(xs)
        torch.ops.akap.car_all_reduce_multi(hs, xs, xs, False)
        torch.cuda.synchronize()
        assert torch.ops.akap.car_error(hs[0]) == 0
        assert (xs[0].float() - exp.float()).abs().max().item() <= 0.05
        assert torch.equal(xs[0], xs[1])
    finally:
        for h in hs:
            torch.ops.akap.car_destroy(h)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _ipc_worker(rank, world, port, q):
    import torch.distributed as dist

    from aws_k8s_ansible_provisioner_amd.parallel.custom_allreduce import CustomAllReduce
    try:
        torch.cuda.set_device(0)
        dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank,
                                world_size=world)
        car = CustomAllReduce(group=None, device=torch.device("cuda", 0), max_bytes=1 << 20)
        res = []
        for it in range(3):
            g = torch.Generator().manual_seed(10 * it + rank)
            x = torch.randn(20000, generator=g).to(torch.bfloat16)
            y = car.all_reduce(x.to(DEV).contiguous())
            torch.cuda.synchronize()
            res.append(y.cpu())
        err = car.error()
        dist.barrier()
        car.close()
        dist.destroy_process_group()
        q.put((rank, err, [r.float().numpy() for r in res]))
    except Exception as e:  # pragma: no cover - reported to the parent
        q.put((rank, repr(e), None))


def test_custom_allreduce_ipc_two_processes():
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_ipc_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    out = {}
    for _ in range(2):
        rank, err, res = q.get(timeout=240)
        out[rank] = (err, res)
    for p in procs:
        p.join(timeout=60)
    for r in range(2):
        assert out[r][0] == 0, out[r][0]
    for it in range(3):
        xs = [torch.randn(20000, generator=torch.Generator().manual_seed(10 * it + r))
              .to(torch.bfloat16) for r in range(2)]
        exp = _ref_sum(xs).float().numpy()
        import numpy as np
        assert np.array_equal(out[0][1][it], out[1][1][it])
        assert np.abs(out[0][1][it] - exp).max() <= 0.05


@pytest.mark.parametrize("world", [2, 4, 8])
@pytest.mark.parametrize("two_shot", [False, True])
@pytest.mark.parametrize("M,d", [(1, 512), (37, 1024), (64, 8192)])
def test_custom_allreduce_resnorm_epilogue(world, two_shot, M, d):
    """All-reduce of row-parallel partial sums fused with the TP decode chain's residual
    epilogue: residual += sum, aout = residual * ln, ss += row sums of residual^2 -- checked
    against fp32 references, identical on every rank (fixed summation order)."""
    ops.load_native(required=True)
    n = M * d
    hs = [torch.ops.akap.car_create(0, r, world, 1 << 20) for r in range(world)]
    try:
        for h in hs:
            torch.ops.akap.car_link_local(h, hs)
        for it in range(2):
            torch.manual_seed(7 * it + world + n)
            xs = [torch.randn(n, dtype=torch.bfloat16, device=DEV) * 0.3 for _ in range(world)]
            res0 = torch.randn(M, d, dtype=torch.bfloat16, device=DEV)
            ln = (torch.rand(d, device=DEV) + 0.5).to(torch.bfloat16)
            res = [res0.clone() for _ in range(world)]
            aout = [torch.empty(M, d, dtype=torch.bfloat16, device=DEV) for _ in range(world)]
            ss = [torch.zeros(M, device=DEV) for _ in range(world)]
            outs = [torch.empty_like(x) for x in xs]  # unused by the epilogue form
            epi = []
            for r in range(world):
                epi += [res[r], ln, aout[r], ss[r]]
            torch.ops.akap.car_all_reduce_multi(hs, xs, outs, two_shot, epi)
            torch.cuda.synchronize()
            assert all(torch.ops.akap.car_error(h) == 0 for h in hs)
            s = (_ref_sum(xs).float().view(M, d) + res0.float()).to(torch.bfloat16)
            for r in range(world):
                assert torch.equal(res[r], res[0]) and torch.equal(aout[r], aout[0])
                assert torch.allclose(ss[r], ss[0])
            assert (res[0].float() - s.float()).abs().max().item() <= 0.05 * world
            assert (aout[0].float() - res[0].float() * ln.float()).abs().max().item() <= \
                0.02 * aout[0].float().abs().max().item()
            assert torch.allclose(ss[0], res[0].float().pow(2).sum(-1), rtol=1e-3, atol=1e-2)
    finally:
        torch.cuda.synchronize()
        for h in hs:
            torch.ops.akap.car_destroy(h)


def _ipc_siblings_worker(rank, world, port, q):
    """All-reduce, all-gather and broadcast launches interleaved on one communicator (the
    per-block epochs are shared by every kind), across `world` processes on one GPU."""
    import torch.distributed as dist

    from aws_k8s_ansible_provisioner_amd.parallel.custom_allreduce import CustomAllReduce
    try:
        torch.cuda.set_device(0)
        dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank,
                                world_size=world)
        car = CustomAllReduce(group=None, device=torch.device("cuda", 0), max_bytes=1 << 20)
        res = []
        for it in range(4):
            g = torch.Generator().manual_seed(100 * it + rank)
            cols = 136 * (40 if it == 3 else 1)
            shard = torch.randn(37, cols, generator=g).to(torch.bfloat16).to(DEV)
            out = torch.empty(37, cols * world, dtype=torch.bfloat16, device=DEV)
            car.all_gather(shard, out)
            x = torch.randn(4096, generator=g).to(torch.bfloat16).to(DEV)
            car.all_reduce(x)
            # broadcast of a uint8 staging region from rank 0 (every rank starts different)
            b = torch.full((2048 + 16 * it,), rank + 1, dtype=torch.uint8, device=DEV)
            if rank == 0:
                b.copy_(torch.arange(b.numel(), dtype=torch.int64).remainder(251).to(torch.uint8))
            car.broadcast(b, 0)
            # equal-segment all-to-all: segment d of rank r holds r * 1000 + d * 10 + j % 7
            # (it 3: several unrolled trips per block plus a ragged tail)
            seg = 24 * (it + 1) + (40000 if it == 3 else 0)
            send = torch.cat([(torch.arange(seg) % 7 + rank * 1000 + d * 10).float()
                              for d in range(world)]).to(torch.bfloat16).to(DEV)
            recv = torch.empty_like(send)
            car.all_to_all(send, recv)
            torch.cuda.synchronize()
            res.append((out.float().cpu().numpy(), b.cpu().numpy(), recv.float().cpu().numpy()))
        err = car.error()
        dist.barrier()
        car.close()
        dist.destroy_process_group()
        q.put((rank, err, res))
    except Exception as e:  # pragma: no cover - reported to the parent
        import traceback
        q.put((rank, repr(e) + traceback.format_exc(), None))


@pytest.mark.parametrize("world", [2, 4])
def test_custom_allgather_broadcast_alltoall_ipc_processes(world):
    """The IPC all-gather (rank-major columns), broadcast and all-to-all, siblings of K13,
    across processes sharing one MI355X: exact against the host-side expectation, every rank."""
    import numpy as np
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_ipc_siblings_worker, args=(r, world, port, q))
             for r in range(world)]
    for p in procs:
        p.start()
    out = {}
    for _ in range(world):
        rank, err, res = q.get(timeout=240)
        out[rank] = (err, res)
    for p in procs:
        p.join(timeout=60)
    for r in range(world):
        assert out[r][0] == 0, out[r][0]
    for it in range(4):
        cols = 136 * (40 if it == 3 else 1)
        shards = [torch.randn(37, cols, generator=torch.Generator().manual_seed(100 * it + r))
                  .to(torch.bfloat16).float().numpy() for r in range(world)]
        want = np.concatenate(shards, axis=1)
        bexp = (np.arange(2048 + 16 * it) % 251).astype(np.uint8)
        seg = 24 * (it + 1) + (40000 if it == 3 else 0)
        for r in range(world):
            got, b, a2a = out[r][1][it]
            assert np.array_equal(got, want), (r, it)
            assert np.array_equal(b, bexp), (r, it)
            # segment p of rank r's result is rank p's segment r
            exp = np.concatenate([(np.arange(seg) % 7 + p * 1000 + r * 10) for p in range(world)])
            assert np.array_equal(a2a, torch.tensor(exp).float().bfloat16().float().numpy()), (r, it)


def _kv_pull_worker(rank, port, q, geo, fp8=False):
    """Rank 0 = prefill: a KV cache with a known pattern, exported by hipIpc.  Rank 1 =
    decode: maps it and pulls blocks + V tails with ONE kv_pull launch."""
    import base64

    import torch.distributed as dist

    from aws_k8s_ansible_provisioner_amd import ops
    try:
        torch.cuda.set_device(0)
        dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank,
                                world_size=2)
        L, Hkv, BS, D, NB0, NB1 = geo
        be = Hkv * BS * D
        if fp8:  # e4m3 cache bytes, moved as bf16 pairs (no V tail)
            be //= 2
        if rank == 0:
            g = torch.Generator().manual_seed(5)
            if fp8:
                kv = torch.randint(0, 256, (L, 2, NB0, 2 * be), generator=g,
                                   dtype=torch.uint8).to(DEV).view(torch.bfloat16)
            else:
                kv = torch.randn(L, 2, NB0, be, generator=g).to(torch.bfloat16).to(DEV)
            planes = kv.view(2 * L, NB0, be)
            meta = [ops.ipc_export(planes), planes.stride(0)]
            dist.broadcast_object_list(meta, src=0)
            dist.barrier()  # rank 1 pulled
            q.put((0, 0, None))
        else:
            meta = [None, None]
            dist.broadcast_object_list(meta, src=0)
            kv = torch.zeros(L, 2, NB1, be, dtype=torch.bfloat16, device=DEV)
            planes = kv.view(2 * L, NB1, be)
            tail = torch.zeros(L, 6, Hkv, 8, D, dtype=torch.bfloat16, device=DEV)
            ptr = ops.ipc_open(meta[0], 0)
            pairs = [(3, 0), (NB0 - 1, 5), (0, NB1 - 1)]
            jobs = [] if fp8 else [(7, 1, 5, 2), (NB0 - 1, BS // 8 - 1, 3, 5)]
            # the peer's planes as a device-address table; our cache as two segments (layer 0,
            # layers 1..) -- the cache of a large engine is several allocations
            src = [ptr + i * meta[1] * 2 for i in range(2 * L)]
            ops.kv_pull(src, NB0, [planes[:2], planes[2:]], pairs, Hkv, BS, D, tail=tail,
                        tail_jobs=jobs)
            torch.cuda.synchronize()
            res = ((kv.view(torch.uint8) if fp8 else kv.float()).cpu().numpy(),
                   tail.float().cpu().numpy())
            ops.ipc_close(ptr)
            dist.barrier()
            q.put((1, 0, res))
        dist.destroy_process_group()
    except Exception as e:  # pragma: no cover - reported to the parent
        import traceback
        q.put((rank, repr(e) + traceback.format_exc(), None))


@pytest.mark.parametrize("fp8", [False, True])
def test_kv_pull_ipc_two_processes(fp8):
    """P/D hipIpc transport: the decode process maps the prefill process's cache and one
    kv_pull launch copies whole blocks (every plane) into its own block ids and writes the
    requests' partial last V groups token-major into their tails -- exact, vs host indexing.
    fp8: an e4m3 (byte) cache, moved as bf16 pairs, blocks only."""
    import numpy as np
    import torch.multiprocessing as mp
    geo = (3, 2, 32, 128, 12, 9)  # L, Hkv, BS, D, prefill blocks, decode blocks
    L, Hkv, BS, D, NB0, NB1 = geo
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_kv_pull_worker, args=(r, port, q, geo, fp8))
             for r in range(2)]
    for p in procs:
        p.start()
    out = {}
    for _ in range(2):
        rank, err, res = q.get(timeout=240)
        out[rank] = (err, res)
    for p in procs:
        p.join(timeout=60)
    assert out[0][0] == 0 and out[1][0] == 0, (out[0][0], out[1][0])
    kv, tail = out[1][1]
    be = Hkv * BS * D
    if fp8:
        src = torch.randint(0, 256, (L, 2, NB0, be), generator=torch.Generator().manual_seed(5),
                            dtype=torch.uint8).numpy()
        want = np.zeros((L, 2, NB1, be), np.uint8)
        for s, d in [(3, 0), (NB0 - 1, 5), (0, NB1 - 1)]:
            want[:, :, d] = src[:, :, s]
        assert np.array_equal(kv, want)
        return
    src = torch.randn(L, 2, NB0, be, generator=torch.Generator().manual_seed(5)) \
        .to(torch.bfloat16).float().numpy()
    want = np.zeros((L, 2, NB1, be), np.float32)
    for s, d in [(3, 0), (NB0 - 1, 5), (0, NB1 - 1)]:
        want[:, :, d] = src[:, :, s]
    assert np.array_equal(kv, want)
    tw = np.zeros((L, 6, Hkv, 8, D), np.float32)
    for s, grp, cnt, slot in [(7, 1, 5, 2), (NB0 - 1, BS // 8 - 1, 3, 5)]:
        v = src[:, 1, s].reshape(L, Hkv, BS // 8, D, 8)[:, :, grp]   # [L, Hkv, D, 8]
        tw[:, slot, :, :cnt] = v[..., :cnt].transpose(0, 1, 3, 2)
    assert np.array_equal(tail, tw)


def _mixed_stress_worker(rank, world, port, q, iters):
    """Back-to-back all-reduces of three sizes (one-shot, two-shot), all-to-alls, broadcasts
    and all-gathers on one communicator with NO host synchronisation between them: every
    launch runs the full grid, so each block's epoch counts every launch and no region is
    restaged while a peer block still reads it (a 1-block launch followed by a
    many-block one of another kind).  Integer-valued inputs make every sum exact."""
    import torch.distributed as dist

    from aws_k8s_ansible_provisioner_amd.parallel.custom_allreduce import CustomAllReduce
    try:
        torch.cuda.set_device(0)
        dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank,
                                world_size=world)
        car = CustomAllReduce(group=None, device=torch.device("cuda", 0), max_bytes=1 << 20)
        keep = []
        for it in range(iters):
            g = torch.Generator().manual_seed(1000 * it + rank)
            for n in (64, 20000, 300000):  # ~1 block, many blocks, two-shot when world > 2
                x = torch.randint(-8, 9, (n,), generator=g).to(torch.bfloat16).to(DEV)
                keep.append(car.all_reduce(x).clone())
            seg = 8 * (1 + it % 5)
            send = torch.randint(-8, 9, (world * seg,), generator=g).to(torch.bfloat16).to(DEV)
            recv = torch.empty_like(send)
            keep.append(car.all_to_all(send, recv).clone())
            b = torch.randint(0, 255, (16 * (1 + it % 7),), generator=g).to(torch.uint8).to(DEV)
            keep.append(car.broadcast(b, it % world).clone())
            shard = torch.randint(-8, 9, (3, 40), generator=g).to(torch.bfloat16).to(DEV)
            out = torch.empty(3, 40 * world, dtype=torch.bfloat16, device=DEV)
            keep.append(car.all_gather(shard, out).clone())
        torch.cuda.synchronize()
        err = car.error()
        res = [k.float().cpu().numpy() for k in keep]
        dist.barrier()
        car.close()
        dist.destroy_process_group()
        q.put((rank, err, res))
    except Exception as e:  # pragma: no cover - reported to the parent
        import traceback
        q.put((rank, repr(e) + traceback.format_exc(), None))


@pytest.mark.parametrize("world", [2, 4])
def test_custom_collectives_mixed_sequence_no_sync(world):
    import numpy as np
    import torch.multiprocessing as mp
    iters = 12
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_mixed_stress_worker, args=(r, world, port, q, iters))
             for r in range(world)]
    for p in procs:
        p.start()
    out = {}
    for _ in range(world):
        rank, err, res = q.get(timeout=240)
        out[rank] = (err, res)
    for p in procs:
        p.join(timeout=60)
    for r in range(world):
        assert out[r][0] == 0, out[r][0]
    # replay every rank's generator on the host
    gens = [torch.Generator().manual_seed(0) for _ in range(world)]
    k = 0
    for it in range(iters):
        for r in range(world):
            gens[r].manual_seed(1000 * it + r)
        for n in (64, 20000, 300000):
            xs = [torch.randint(-8, 9, (n,), generator=gens[r]).float() for r in range(world)]
            want = sum(xs).numpy()
            for r in range(world):
                assert np.array_equal(out[r][1][k], want), ("all_reduce", it, n, r)
            k += 1
        seg = 8 * (1 + it % 5)
        sends = [torch.randint(-8, 9, (world * seg,), generator=gens[r]).float().numpy()
                 for r in range(world)]
        for r in range(world):
            want = np.concatenate([sends[p][r * seg:(r + 1) * seg] for p in range(world)])
            assert np.array_equal(out[r][1][k], want), ("all_to_all", it, r)
        k += 1
        bs = [torch.randint(0, 255, (16 * (1 + it % 7),), generator=gens[r]).numpy()
              for r in range(world)]
        for r in range(world):
            assert np.array_equal(out[r][1][k], bs[it % world].astype(np.float32)), ("bcast", it)
        k += 1
        shards = [torch.randint(-8, 9, (3, 40), generator=gens[r]).float().numpy()
                  for r in range(world)]
        for r in range(world):
            assert np.array_equal(out[r][1][k], np.concatenate(shards, axis=1)), ("gather", it)
        k += 1
