// Minimal HIP-only reproducer for the hipGraph stream-capture segfault seen from PyTorch
// (profiles/r1_decode_overlap_experiment.log: bench/graph_multistream_probe.py pingpong / alt 28).
// No PyTorch: plain hipStreamBeginCapture on a main stream, cross-stream dependencies by
// hipEventRecord + hipStreamWaitEvent (what torch.cuda.Stream.wait_stream does), a trivial
// kernel per node.  A SIGSEGV handler prints the native backtrace.
//
//   hipcc --offload-arch=gfx950 -O1 -g bench/graph_capture_repro.hip -o /tmp/gcr
//   /tmp/gcr <pattern> <n> [reuse_events]
// patterns:
//   fork     main -> {s1, s2} -> main                            (control)
//   pingpong s1 -> s2 -> s1 -> s2 ... (n hops), the two streams reused every hop
//   fresh    the same chain, but every hop continues on a NEW stream
//   alt      two chains on streams that are replaced by fresh streams at every hop, each new
//            stream also waiting on the other chain's latest event (the overlap pattern)
// reuse_events=1: one event per stream re-recorded every hop (torch allocates a new one per
// wait_stream; both are tried)
#include <execinfo.h>
#include <hip/hip_runtime.h>
#include <signal.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <unistd.h>

#include <string>
#include <vector>

#define CK(x)                                                                     \
  do {                                                                            \
    hipError_t e_ = (x);                                                          \
    if (e_ != hipSuccess) {                                                       \
      fprintf(stderr, "%s:%d %s -> %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
      exit(2);                                                                    \
    }                                                                             \
  } while (0)

__global__ void axpb(float* y, const float* x, float a, float b, int n) {
  int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) y[i] = a * x[i] + b;
}

static void on_segv(int sig) {
  void* f[64];
  const int n = backtrace(f, 64);
  const char msg[] = "\n*** SIGSEGV during capture; native backtrace:\n";
  (void)!write(2, msg, sizeof(msg) - 1);
  backtrace_symbols_fd(f, n, 2);
  _exit(139);
}

static bool reuse_events = false;
static std::vector<hipEvent_t> all_events;

static hipEvent_t new_event() {
  hipEvent_t e;
  CK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
  all_events.push_back(e);
  return e;
}

// torch's Stream.wait_stream(other): record a fresh event on `other`, make `s` wait on it
static void wait_stream(hipStream_t s, hipStream_t other, hipEvent_t* cached) {
  hipEvent_t e = (reuse_events && cached) ? *cached : new_event();
  if (reuse_events && cached && *cached == nullptr) e = *cached = new_event();
  CK(hipEventRecord(e, other));
  CK(hipStreamWaitEvent(s, e, 0));
}

int main(int argc, char** argv) {
  signal(SIGSEGV, on_segv);
  const std::string pat = argc > 1 ? argv[1] : "pingpong";
  const int n = argc > 2 ? atoi(argv[2]) : 2;
  reuse_events = argc > 3 && atoi(argv[3]) != 0;
  const int N = 1 << 16;
  std::vector<float*> buf(4 * n + 8);
  for (auto& b : buf) CK(hipMalloc(&b, N * sizeof(float)));
  hipStream_t main_s, s1, s2;
  CK(hipStreamCreateWithFlags(&main_s, hipStreamNonBlocking));
  CK(hipStreamCreateWithFlags(&s1, hipStreamNonBlocking));
  CK(hipStreamCreateWithFlags(&s2, hipStreamNonBlocking));
  std::vector<hipStream_t> pool(4 * n + 8);
  for (auto& s : pool) CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  hipEvent_t c1 = nullptr, c2 = nullptr;
  auto k = [&](hipStream_t s, int out, int in) {
    axpb<<<N / 256, 256, 0, s>>>(buf[out], buf[in], 1.0001f, 0.001f, N);
    CK(hipGetLastError());
  };
  printf("capturing %s n=%d reuse_events=%d\n", pat.c_str(), n, (int)reuse_events);
  fflush(stdout);
  hipGraph_t g;
  CK(hipStreamBeginCapture(main_s, hipStreamCaptureModeGlobal));
  k(main_s, 0, 1);
  if (pat == "fork") {
    wait_stream(s1, main_s, nullptr);
    wait_stream(s2, main_s, nullptr);
    k(s1, 2, 0);
    k(s2, 3, 0);
    wait_stream(main_s, s1, nullptr);
    wait_stream(main_s, s2, nullptr);
  } else if (pat == "pingpong") {
    wait_stream(s1, main_s, nullptr);
    wait_stream(s2, main_s, nullptr);
    int cur = 0;
    for (int i = 0; i < n; ++i) {
      k(s1, 2 + 2 * i, cur);
      wait_stream(s2, s1, &c1);
      k(s2, 3 + 2 * i, 2 + 2 * i);
      cur = 3 + 2 * i;
      wait_stream(s1, s2, &c2);
    }
    wait_stream(main_s, s1, nullptr);
    wait_stream(main_s, s2, nullptr);
  } else if (pat == "pingpong_nojoin2") {
    // same chain, but s2 is NOT joined back into main explicitly (s1 already waits on it)
    wait_stream(s1, main_s, nullptr);
    wait_stream(s2, main_s, nullptr);
    int cur = 0;
    for (int i = 0; i < n; ++i) {
      k(s1, 2 + 2 * i, cur);
      wait_stream(s2, s1, &c1);
      k(s2, 3 + 2 * i, 2 + 2 * i);
      cur = 3 + 2 * i;
      wait_stream(s1, s2, &c2);
    }
    wait_stream(main_s, s1, nullptr);
  } else if (pat == "fresh") {
    hipStream_t prev = main_s;
    int cur = 0;
    for (int i = 0; i < n; ++i) {
      hipStream_t a = pool[2 * i], b = pool[2 * i + 1];
      wait_stream(a, prev, nullptr);
      k(a, 2 + 2 * i, cur);
      wait_stream(b, a, nullptr);
      k(b, 3 + 2 * i, 2 + 2 * i);
      cur = 3 + 2 * i;
      prev = b;
    }
    wait_stream(main_s, prev, nullptr);
  } else if (pat == "alt") {
    hipStream_t cur[2] = {pool[0], pool[1]};
    wait_stream(cur[0], main_s, nullptr);
    wait_stream(cur[1], main_s, nullptr);
    int used = 2;
    hipEvent_t last = nullptr;
    int y[2] = {0, 0};
    for (int i = 0; i < n; ++i) {
      for (int c = 0; c < 2; ++c) {
        if (last != nullptr) {
          hipStream_t ns = pool[used++ % pool.size()];
          wait_stream(ns, cur[c], nullptr);
          CK(hipStreamWaitEvent(ns, last, 0));
          cur[c] = ns;
        }
        const int o = 2 + (4 * i + 2 * c) % (int)(buf.size() - 2);
        k(cur[c], o, y[c]);
        last = new_event();
        CK(hipEventRecord(last, cur[c]));
        k(cur[c], o + 1, o);
        y[c] = o + 1;
      }
    }
    wait_stream(main_s, cur[0], nullptr);
    wait_stream(main_s, cur[1], nullptr);
  } else {
    fprintf(stderr, "unknown pattern\n");
    return 2;
  }
  CK(hipStreamEndCapture(main_s, &g));
  size_t nodes = 0;
  CK(hipGraphGetNodes(g, nullptr, &nodes));
  printf("captured: %zu nodes\n", nodes);
  fflush(stdout);
  hipGraphExec_t ge;
  CK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
  CK(hipGraphLaunch(ge, main_s));
  CK(hipStreamSynchronize(main_s));
  printf("replayed ok\n");
  return 0;
}
