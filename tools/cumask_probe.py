"""Probe: do hipExtStreamCreateWithCUMask stream masks survive hipGraph capture, and can a
CU-partitioned pair of streams overlap an HBM-streaming kernel with latency-bound GEMMs?

  python tools/cumask_probe.py
"""
import ctypes
import os

import torch

lib = ctypes.CDLL(os.path.join(os.path.dirname(torch.__file__), "lib", "libamdhip64.so"))


def masked(cus):
    words = [0] * 8
    for c in cus:
        words[c // 32] |= 1 << (c % 32)
    s = ctypes.c_void_p()
    arr = (ctypes.c_uint32 * 8)(*words)
    rc = lib.hipExtStreamCreateWithCUMask(ctypes.byref(s), ctypes.c_uint32(8), arr)
    assert rc == 0, f"hipExtStreamCreateWithCUMask -> {rc}"
    return torch.cuda.ExternalStream(s.value)


def timed(fn, stream, reps=5):
    with torch.cuda.stream(stream):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(True), torch.cuda.Event(True)
    e0.record(stream)
    with torch.cuda.stream(stream):
        for _ in range(reps):
            fn()
    e1.record(stream)
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps * 1000


def graph_of(fn, stream):
    with torch.cuda.stream(stream):
        fn()
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=stream):
        fn()
    return g


def main():
    torch.cuda.init()
    n = torch.cuda.get_device_properties(0).multi_processor_count
    dflt = torch.cuda.current_stream()
    x = torch.randn(8192, 8192, device="cuda", dtype=torch.bfloat16)
    mm = lambda: torch.mm(x, x)  # noqa: E731
    m8 = masked(range(8))
    t_full = timed(mm, dflt)
    t_m8 = timed(mm, m8)
    g = graph_of(mm, m8)
    t_g8 = timed(g.replay, m8)
    t_g8d = timed(g.replay, dflt)
    print(f"[mask] {n} CUs; 8192^3 bf16 mm: full {t_full:.0f} us, 8-CU stream eager {t_m8:.0f} us, "
          f"graph captured on it replayed on it {t_g8:.0f} us / on the default stream "
          f"{t_g8d:.0f} us", flush=True)

    # overlap: HBM stream (elementwise over 2 GiB) vs a chain of 28 x 4 decode-size GEMMs
    big = torch.randn(1 << 30, device="cuda", dtype=torch.bfloat16)
    out = torch.empty_like(big)
    a = torch.randn(256, 1024, device="cuda", dtype=torch.bfloat16)
    ws = [torch.randn(4096, 1024, device="cuda", dtype=torch.bfloat16),
          torch.randn(1024, 2048, device="cuda", dtype=torch.bfloat16),
          torch.randn(6144, 1024, device="cuda", dtype=torch.bfloat16),
          torch.randn(1024, 3072, device="cuda", dtype=torch.bfloat16)]
    stream_fn = lambda: torch.mul(big, 1.0001, out=out)  # noqa: E731

    def chain():
        for _ in range(28):
            torch.nn.functional.linear(a, ws[0])
            torch.nn.functional.linear(torch.empty(256, 2048, device="cuda",
                                                   dtype=torch.bfloat16), ws[1])
            torch.nn.functional.linear(a, ws[2])
            torch.nn.functional.linear(torch.empty(256, 3072, device="cuda",
                                                   dtype=torch.bfloat16), ws[3])

    # every workload captured in a hipGraph (eager launches of 112 GEMMs are host-bound); a graph
    # runs on the CUs of the stream it is launched on
    g_chain = graph_of(chain, torch.cuda.Stream())
    g_strm = graph_of(stream_fn, torch.cuda.Stream())
    t_s = timed(g_strm.replay, dflt)
    t_c = timed(g_chain.replay, dflt)
    print(f"[overlap] graphs on the full chip: stream 4 GiB moved {t_s:.0f} us "
          f"({4.29e9 / t_s / 1e6:.2f} TB/s); 112-GEMM M=256 chain {t_c:.0f} us", flush=True)
    for k in (16, 32, 64, 96):
        sg, ss = masked(range(k)), masked(range(k, n))
        tc_k = timed(g_chain.replay, sg)
        ts_k = timed(g_strm.replay, ss)
        reps_s = max(1, round(3 * t_c / t_s))  # the stream side ~3x the chain (attention : GEMMs)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(True), torch.cuda.Event(True)
        e0.record(dflt)
        sg.wait_stream(dflt)
        ss.wait_stream(dflt)
        with torch.cuda.stream(sg):
            g_chain.replay()
        with torch.cuda.stream(ss):
            for _ in range(reps_s):
                g_strm.replay()
        dflt.wait_stream(sg)
        dflt.wait_stream(ss)
        e1.record(dflt)
        torch.cuda.synchronize()
        both = e0.elapsed_time(e1) * 1000
        print(f"[overlap] k={k:3d}: chain on {k} CUs {tc_k:.0f} us, stream on {n - k} CUs "
              f"{ts_k:.0f} us; chain || {reps_s} streams {both:.0f} us vs serial on the full "
              f"chip {t_c + reps_s * t_s:.0f} us", flush=True)


if __name__ == "__main__":
    main()
