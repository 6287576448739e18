// hipIpc import reproducer, HIP runtime only (no torch, no RCCL): does opening a peer process's
// exported device memory hang, and what triggers it?  (the P/D rehearsals
// saw hipIpcOpenMemHandle of a 79-101 GiB peer KV cache hang once the importing process held
// most of the device, profiles/r5 "hipIpc multi-importer hang")
//
//   ipc_import_repro export <Y_GiB> <seg_GiB> <dir> [importers]
//       allocate Y GiB as ceil(Y / seg) device allocations (the KV exporter's <= 32 GiB
//       segments, parallel/kv_transfer.py), fill each, write their hipIpcMemHandles to
//       <dir>/handles.bin, then wait (<= 70 s) for every importer's <dir>/done.<id> and exit
//   ipc_import_repro import <X_GiB> <dir> [id] [fill] [piece_GiB]
//       allocate and hold X GiB of its own first (piece_GiB pieces, default 16; 0 = one
//       allocation, as PyTorch's allocator makes for one big tensor; fill = 1: also write them,
//       as a zero-filled KV cache is), wait for the handles, open every segment
//       (hipIpcMemLazyEnablePeerAccess), read 16 bytes of each back, print the free memory
//       and the time of every step, write <dir>/done.<id>.  Several importers of one export =
//       the 1 prefill : 2 decode layout.
// Every line is flushed, so a hang shows as the last step printed.  The sweep driver
// (tools/gpu/s9_ipc_sweep.sh) runs each (X, Y) point under `timeout` and stops at the first
// hang.  Same-device import: both processes run on GPU 0 (the one-GPU P/D rehearsal layout).
//
// The HIP runtime is dlopen'ed from $IPC_REPRO_HIPLIB (default /opt/rocm/lib/libamdhip64.so,
// ROCm 7.2) so the same binary can run on the runtime PyTorch bundles
// (torch/lib/libamdhip64.so, ROCm 7.0.2), which is the one every engine process uses: both
// carry the soname libamdhip64.so.7, so a torch process never loads /opt/rocm's.
// Host-only C++ (no device code): g++ -O2 -std=c++17 ipc_import_repro.cpp -ldl
#include <dlfcn.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <thread>
#include <vector>

// the few runtime entry points used, resolved from the chosen library
typedef int hipError_t;
struct hipIpcMemHandle_t {
  char reserved[64];
};
constexpr unsigned hipIpcMemLazyEnablePeerAccess = 1;
constexpr int hipMemcpyDeviceToHost = 2;
static hipError_t (*hipMalloc)(void**, size_t);
static hipError_t (*hipFree)(void*);
static hipError_t (*hipMemset)(void*, int, size_t);
static hipError_t (*hipDeviceSynchronize)();
static hipError_t (*hipMemGetInfo)(size_t*, size_t*);
static hipError_t (*hipIpcGetMemHandle)(hipIpcMemHandle_t*, void*);
static hipError_t (*hipIpcOpenMemHandle)(void**, hipIpcMemHandle_t, unsigned);
static hipError_t (*hipMemcpy)(void*, const void*, size_t, int);
static const char* (*hipGetErrorString)(hipError_t);
static hipError_t (*hipRuntimeGetVersion)(int*);

static void load_runtime() {
  const char* path = std::getenv("IPC_REPRO_HIPLIB");
  if (path == nullptr) path = "/opt/rocm/lib/libamdhip64.so";
  void* h = dlopen(path, RTLD_NOW | RTLD_LOCAL);
  if (h == nullptr) {
    std::printf("dlopen %s: %s\n", path, dlerror());
    std::exit(8);
  }
  auto sym = [&](const char* n) {
    void* f = dlsym(h, n);
    if (f == nullptr) {
      std::printf("missing %s in %s\n", n, path);
      std::exit(8);
    }
    return f;
  };
  hipMalloc = reinterpret_cast<decltype(hipMalloc)>(sym("hipMalloc"));
  hipFree = reinterpret_cast<decltype(hipFree)>(sym("hipFree"));
  hipMemset = reinterpret_cast<decltype(hipMemset)>(sym("hipMemset"));
  hipDeviceSynchronize = reinterpret_cast<decltype(hipDeviceSynchronize)>(sym("hipDeviceSynchronize"));
  hipMemGetInfo = reinterpret_cast<decltype(hipMemGetInfo)>(sym("hipMemGetInfo"));
  hipIpcGetMemHandle = reinterpret_cast<decltype(hipIpcGetMemHandle)>(sym("hipIpcGetMemHandle"));
  hipIpcOpenMemHandle = reinterpret_cast<decltype(hipIpcOpenMemHandle)>(sym("hipIpcOpenMemHandle"));
  hipMemcpy = reinterpret_cast<decltype(hipMemcpy)>(sym("hipMemcpy"));
  hipGetErrorString = reinterpret_cast<decltype(hipGetErrorString)>(sym("hipGetErrorString"));
  hipRuntimeGetVersion = reinterpret_cast<decltype(hipRuntimeGetVersion)>(sym("hipRuntimeGetVersion"));
  int v = 0;
  hipRuntimeGetVersion(&v);
  std::printf("[runtime] %s, HIP runtime version %d\n", path, v);
  std::fflush(stdout);
}

#define CHECK(x)                                                                       \
  do {                                                                                 \
    hipError_t e_ = (x);                                                               \
    if (e_ != 0) {                                                                     \
      std::printf("HIP error %s at %s:%d (%s)\n", hipGetErrorString(e_), __FILE__,     \
                  __LINE__, #x);                                                       \
      std::fflush(stdout);                                                             \
      std::exit(3);                                                                    \
    }                                                                                  \
  } while (0)

static const auto T0 = std::chrono::steady_clock::now();

static double secs() {
  return std::chrono::duration<double>(std::chrono::steady_clock::now() - T0).count();
}

static void say(const char* role, const std::string& msg) {
  size_t fr = 0, tot = 0;
  (void)hipMemGetInfo(&fr, &tot);
  std::printf("[%s +%.2fs free %.1f/%.1f GiB] %s\n", role, secs(), fr / 1073741824.0,
              tot / 1073741824.0, msg.c_str());
  std::fflush(stdout);
}

static bool exists(const std::string& p) {
  FILE* f = std::fopen(p.c_str(), "rb");
  if (f) std::fclose(f);
  return f != nullptr;
}

static int done_count(const std::string& dir, int nimp) {
  int c = 0;
  for (int i = 0; i < nimp; ++i) c += exists(dir + "/done." + std::to_string(i));
  return c;
}

static int do_export(double y_gib, double seg_gib, const std::string& dir, int nimp) {
  const size_t total = (size_t)(y_gib * 1073741824.0), seg = (size_t)(seg_gib * 1073741824.0);
  std::vector<void*> ptrs;
  std::vector<hipIpcMemHandle_t> hs;
  for (size_t off = 0; off < total; off += seg) {
    const size_t n = total - off < seg ? total - off : seg;
    void* p = nullptr;
    CHECK(hipMalloc(&p, n));
    CHECK(hipMemset(p, 0x5a, n));
    hipIpcMemHandle_t h;
    CHECK(hipIpcGetMemHandle(&h, p));
    ptrs.push_back(p);
    hs.push_back(h);
  }
  CHECK(hipDeviceSynchronize());
  say("export", "allocated and filled " + std::to_string(ptrs.size()) + " segment(s), " +
                    std::to_string(y_gib) + " GiB");
  const std::string tmp = dir + "/handles.tmp", fin = dir + "/handles.bin";
  FILE* f = std::fopen(tmp.c_str(), "wb");
  if (!f) return 4;
  const int n = (int)hs.size();
  std::fwrite(&n, sizeof n, 1, f);
  for (auto& h : hs) std::fwrite(&h, sizeof h, 1, f);
  for (size_t i = 0; i < ptrs.size(); ++i) {  // segment sizes
    const size_t sz = total - i * seg < seg ? total - i * seg : seg;
    std::fwrite(&sz, sizeof sz, 1, f);
  }
  std::fclose(f);
  std::rename(tmp.c_str(), fin.c_str());
  say("export", "handles published");
  for (int i = 0; i < 700 && done_count(dir, nimp) < nimp; ++i)  // <= 70 s
    std::this_thread::sleep_for(std::chrono::milliseconds(100));
  say("export", done_count(dir, nimp) == nimp ? "importers done" : "gave up waiting");
  for (void* p : ptrs) CHECK(hipFree(p));
  return 0;
}

static int do_import(double x_gib, const std::string& dir, int id, bool fill, double piece_gib) {
  std::vector<void*> own;
  const size_t hold = (size_t)(x_gib * 1073741824.0);
  const size_t piece = piece_gib > 0 ? (size_t)(piece_gib * 1073741824.0) : (hold ? hold : 1);
  for (size_t off = 0; off < hold; off += piece) {
    void* p = nullptr;
    const size_t n = hold - off < piece ? hold - off : piece;
    CHECK(hipMalloc(&p, n));
    if (fill) CHECK(hipMemset(p, 0, n));
    own.push_back(p);
  }
  CHECK(hipDeviceSynchronize());
  say("import", "holding " + std::to_string(x_gib) + " GiB of its own");
  const std::string fin = dir + "/handles.bin";
  for (int i = 0; i < 1200 && !exists(fin); ++i)
    std::this_thread::sleep_for(std::chrono::milliseconds(100));
  FILE* f = std::fopen(fin.c_str(), "rb");
  if (!f) {
    say("import", "no handles");
    return 5;
  }
  int n = 0;
  if (std::fread(&n, sizeof n, 1, f) != 1 || n <= 0 || n > 64) return 6;
  std::vector<hipIpcMemHandle_t> hs(n);
  std::vector<size_t> sz(n);
  for (auto& h : hs)
    if (std::fread(&h, sizeof h, 1, f) != 1) return 6;
  for (auto& s : sz)
    if (std::fread(&s, sizeof s, 1, f) != 1) return 6;
  std::fclose(f);
  double mapped = 0;
  for (int i = 0; i < n; ++i) {
    say("import", "opening segment " + std::to_string(i) + " (" +
                      std::to_string(sz[i] / 1073741824.0) + " GiB)");
    const double t = secs();
    void* p = nullptr;
    CHECK(hipIpcOpenMemHandle(&p, hs[i], hipIpcMemLazyEnablePeerAccess));
    unsigned char b[16];
    CHECK(hipMemcpy(b, static_cast<char*>(p) + sz[i] - 16, 16, hipMemcpyDeviceToHost));
    mapped += sz[i] / 1073741824.0;
    char msg[160];
    std::snprintf(msg, sizeof msg, "opened segment %d in %.3f s, last bytes 0x%02x (want 0x5a)",
                  i, secs() - t, b[15]);
    say("import", msg);
    if (b[15] != 0x5a) return 7;
  }
  char msg[160];
  std::snprintf(msg, sizeof msg, "OK: held %.1f GiB + mapped %.1f GiB of the peer", x_gib, mapped);
  say("import", msg);
  FILE* d = std::fopen((dir + "/done." + std::to_string(id)).c_str(), "wb");
  if (d) std::fclose(d);
  for (void* p : own) CHECK(hipFree(p));
  return 0;
}

int main(int argc, char** argv) {
  if (argc >= 2 && (!std::strcmp(argv[1], "export") || !std::strcmp(argv[1], "import")))
    load_runtime();
  if (argc >= 5 && !std::strcmp(argv[1], "export"))
    return do_export(std::atof(argv[2]), std::atof(argv[3]), argv[4],
                     argc >= 6 ? std::atoi(argv[5]) : 1);
  if (argc >= 4 && !std::strcmp(argv[1], "import"))
    return do_import(std::atof(argv[2]), argv[3], argc >= 5 ? std::atoi(argv[4]) : 0,
                     argc >= 6 && std::atoi(argv[5]) == 1, argc >= 7 ? std::atof(argv[6]) : 16);
  std::fprintf(stderr,
               "usage: %s export <Y_GiB> <seg_GiB> <dir> [importers] | "
               "import <X_GiB> <dir> [id] [fill] [piece_GiB]\n", argv[0]);
  return 2;
}
