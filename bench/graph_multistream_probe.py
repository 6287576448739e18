"""Probe: hipGraph capture of fork/join and ping-pong dependencies across HIP streams.
python bench/graph_multistream_probe.py basic|event|pingpong|pingpong_prealloc [n]"""
import ctypes
import faulthandler
import os
import sys

import torch

faulthandler.enable()
if os.environ.get("AKAP_SEGV_BT"):  # native backtrace on SIGSEGV, then faulthandler's stack
    ctypes.CDLL(os.path.join(os.path.dirname(os.path.abspath(__file__)), "segv_bt.so"))

step = sys.argv[1] if len(sys.argv) > 1 else "basic"
n = int(sys.argv[2]) if len(sys.argv) > 2 else 30
x = torch.randn(1 << 20, device="cuda")
s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()
bufs = [torch.empty_like(x) for _ in range(2 * n + 2)]
POOL = [torch.cuda.Stream() for _ in range(4 * n + 4)]
bufs2 = [torch.empty_like(x) for _ in range(2 * n + 2)]
KEEP = []


def body():
    main = torch.cuda.current_stream()
    s1.wait_stream(main)
    s2.wait_stream(main)
    if step == "fresh":  # every cross-stream hop continues on a brand-new stream
        y = x
        prev = main
        for i in range(n):
            sa = POOL[2 * i]
            sa.wait_stream(prev)
            with torch.cuda.stream(sa):
                torch.mul(y, 1.0001, out=bufs[2 * i])
            sb = POOL[2 * i + 1]
            sb.wait_stream(sa)
            with torch.cuda.stream(sb):
                torch.add(bufs[2 * i], 0.001, out=bufs[2 * i + 1])
            y = bufs[2 * i + 1]
            prev = sb
        main.wait_stream(prev)
        return y
    if step in ("alt", "alt_alloc"):  # run_fresh's pattern: events mid-stream, fresh waiters
        cur = [POOL[0], POOL[1]]
        for c in cur:
            c.wait_stream(main)
        it = iter(POOL[2:])
        ys = [x, x]
        last = None
        for i in range(n):
            for k in range(2):
                if last is not None:
                    ns = next(it)
                    ns.wait_stream(cur[k])
                    ns.wait_event(last)
                    cur[k] = ns
                with torch.cuda.stream(cur[k]):
                    if step == "alt_alloc":
                        ys[k] = ys[k] * 1.0001
                    else:
                        torch.mul(ys[k], 1.0001, out=bufs[(2 * i + k) % len(bufs)])
                        ys[k] = bufs[(2 * i + k) % len(bufs)]
                last = torch.cuda.Event()
                last.record(cur[k])
                KEEP.append(last)
                with torch.cuda.stream(cur[k]):
                    if step == "alt_alloc":
                        ys[k] = ys[k] + 0.001
                    else:
                        torch.add(ys[k], 0.001, out=bufs2[(2 * i + k) % len(bufs2)])
                        ys[k] = bufs2[(2 * i + k) % len(bufs2)]
        for c in cur:
            main.wait_stream(c)
        return ys[0] + ys[1]
    if step.startswith("pingpong"):
        y = x
        for i in range(n):
            with torch.cuda.stream(s1):
                if step == "pingpong_prealloc":
                    torch.mul(y, 1.0001, out=bufs[2 * i])
                    y1 = bufs[2 * i]
                else:
                    y1 = y * 1.0001
            s2.wait_stream(s1)
            with torch.cuda.stream(s2):
                if step == "pingpong_prealloc":
                    torch.add(y1, 0.001, out=bufs[2 * i + 1])
                    y = bufs[2 * i + 1]
                else:
                    y = y1 + 0.001
            s1.wait_stream(s2)
        main.wait_stream(s1)
        main.wait_stream(s2)
        return y
    with torch.cuda.stream(s1):
        a = x * 2
    with torch.cuda.stream(s2):
        b = x + 1
        if step == "event":
            e = torch.cuda.Event()
            e.record(s2)
            s1.wait_event(e)
    main.wait_stream(s1)
    main.wait_stream(s2)
    return a + b


ref = body().clone()
torch.cuda.synchronize()
g = torch.cuda.CUDAGraph()
print("capturing", step, n, flush=True)
with torch.cuda.graph(g):
    y = body()
print("captured", flush=True)
g.replay()
torch.cuda.synchronize()
print("ok", bool(torch.equal(y, ref)), flush=True)
