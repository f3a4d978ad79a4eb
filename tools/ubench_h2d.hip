// Host -> HBM upload rate for the host-input path (odo_track_batch_host):
// page-locked allocations with different hipHostMalloc flags, a registered
// malloc() buffer, and one vs two copy streams, each copying one 256-frame
// 640x480 batch (BGR8 + depth16 = 393 MB) as the library does (BGR then depth).
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>

#define CHECK(x)                                                                           \
  do {                                                                                     \
    hipError_t e_ = (x);                                                                   \
    if (e_ != hipSuccess) {                                                                \
      fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_));   \
      exit(1);                                                                             \
    }                                                                                      \
  } while (0)

static const size_t kPix = (size_t)256 * 640 * 480;
static const size_t kBgr = kPix * 3, kDep = kPix * 2;

static double run(const char* name, unsigned char* h, unsigned char* d, int nstreams, int chunks) {
  hipStream_t st[2];
  for (int i = 0; i < nstreams; i++) CHECK(hipStreamCreateWithFlags(&st[i], hipStreamNonBlocking));
  hipEvent_t a, b;
  CHECK(hipEventCreate(&a));
  CHECK(hipEventCreate(&b));
  auto once = [&]() {
    // BGR then depth, each split in `chunks` pieces round robin over the streams
    size_t parts[2][2] = {{0, kBgr}, {kBgr, kDep}};
    int k = 0;
    for (auto& p : parts) {
      const size_t piece = (p[1] + chunks - 1) / chunks;
      for (size_t o = 0; o < p[1]; o += piece, k++) {
        const size_t n = o + piece > p[1] ? p[1] - o : piece;
        CHECK(hipMemcpyAsync(d + p[0] + o, h + p[0] + o, n, hipMemcpyHostToDevice, st[k % nstreams]));
      }
    }
  };
  once();
  CHECK(hipDeviceSynchronize());
  const int reps = 5;
  CHECK(hipEventRecord(a, st[0]));
  for (int r = 0; r < reps; r++) once();
  for (int i = 1; i < nstreams; i++) {
    hipEvent_t e;
    CHECK(hipEventCreate(&e));
    CHECK(hipEventRecord(e, st[i]));
    CHECK(hipStreamWaitEvent(st[0], e, 0));
  }
  CHECK(hipEventRecord(b, st[0]));
  CHECK(hipEventSynchronize(b));
  float ms = 0;
  CHECK(hipEventElapsedTime(&ms, a, b));
  const double gbs = reps * (double)(kBgr + kDep) / (ms * 1e-3) / 1e9;
  printf("{\"bench\": \"h2d\", \"alloc\": \"%s\", \"streams\": %d, \"chunks\": %d, \"ms_per_batch\": %.3f, "
         "\"gbs\": %.2f}\n", name, nstreams, chunks, ms / reps, gbs);
  fflush(stdout);
  for (int i = 0; i < nstreams; i++) CHECK(hipStreamDestroy(st[i]));
  return gbs;
}

int main() {
  unsigned char* d;
  CHECK(hipMalloc(&d, kBgr + kDep));
  struct { const char* name; unsigned flags; } kinds[] = {
      {"hipHostMallocDefault", hipHostMallocDefault},
      {"hipHostMallocPortable", hipHostMallocPortable},
      {"hipHostMallocWriteCombined", hipHostMallocWriteCombined},
      {"hipHostMallocNonCoherent", hipHostMallocNonCoherent},
      {"hipHostMallocCoherent", hipHostMallocCoherent},
      {"hipHostMallocNumaUser", hipHostMallocNumaUser},
  };
  for (auto& k : kinds) {
    unsigned char* h = nullptr;
    if (hipHostMalloc((void**)&h, kBgr + kDep, k.flags) != hipSuccess) {
      printf("{\"bench\": \"h2d\", \"alloc\": \"%s\", \"error\": \"alloc failed\"}\n", k.name);
      continue;
    }
    memset(h, 7, kBgr + kDep);
    run(k.name, h, d, 1, 1);
    run(k.name, h, d, 2, 2);
    run(k.name, h, d, 2, 8);
    CHECK(hipHostFree(h));
  }
  unsigned char* m = (unsigned char*)aligned_alloc(4096, kBgr + kDep);
  memset(m, 7, kBgr + kDep);
  CHECK(hipHostRegister(m, kBgr + kDep, hipHostRegisterDefault));
  run("malloc+hipHostRegister", m, d, 1, 1);
  run("malloc+hipHostRegister", m, d, 2, 2);
  CHECK(hipHostUnregister(m));
  run("malloc (pageable)", m, d, 1, 1);
  free(m);
  CHECK(hipFree(d));
  return 0;
}
