// HBM ceilings for the sweep's traffic shape (tools only, not part of the engine):
// a 200 MB stream read (the idle sweep) and an in-place 200 MB read + rewrite (the churn
// sweep's state lines), with the sweep's own launch shape (256-thread blocks, 16 B per lane,
// grid-stride tiles); and a write-only stream (the patch emitter's output: what a writer of
// whole lines can reach).  Prints us per launch and TB/s.
//   hipcc --offload-arch=gfx950 -O3 -o tools/hbm_ceiling tools/hbm_ceiling.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <cstdlib>

__global__ __launch_bounds__(256) void read_k(const uint4* __restrict__ p, size_t n, uint32_t* out) {
  uint32_t acc = 0;
  for (size_t i = blockIdx.x * 256ull + threadIdx.x; i < n; i += (size_t)gridDim.x * 256ull) {
    const uint4 v = p[i];
    acc ^= v.x ^ v.y ^ v.z ^ v.w;
  }
  if (acc == 0x12345678u) out[0] = acc;
}

__global__ __launch_bounds__(256) void rw_k(uint4* __restrict__ p, size_t n) {
  for (size_t i = blockIdx.x * 256ull + threadIdx.x; i < n; i += (size_t)gridDim.x * 256ull) {
    uint4 v = p[i];
    v.x ^= 1u;
    typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
    __builtin_nontemporal_store(u32x4{v.x, v.y, v.z, v.w}, reinterpret_cast<u32x4*>(p + i));
  }
}

__global__ __launch_bounds__(256) void write_k(uint4* __restrict__ p, size_t n) {
  for (size_t i = blockIdx.x * 256ull + threadIdx.x; i < n; i += (size_t)gridDim.x * 256ull)
    p[i] = make_uint4((uint32_t)i, 1u, 2u, 3u);
}

int main(int argc, char** argv) {
  const size_t bytes = (argc > 1 ? (size_t)atoll(argv[1]) : 200ull) << 20, n = bytes / 16;
  printf("buffer %zu MiB\n", bytes >> 20);
  uint4* p;
  uint32_t* o;
  hipMalloc(&p, bytes);
  hipMalloc(&o, 4);
  hipMemset(p, 1, bytes);
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  const int grids[] = {1024, 2048, 4096, 8192, 16384, (int)((n + 255) / 256)};
  for (int g : grids) {
    for (int kind = 0; kind < 3; ++kind) {
      auto run = [&]() {
        if (kind == 0) read_k<<<g, 256>>>(p, n, o);
        else if (kind == 1) rw_k<<<g, 256>>>(p, n);
        else write_k<<<g, 256>>>(p, n);
      };
      for (int w = 0; w < 3; ++w) run();
      hipEventRecord(a);
      const int reps = 20;
      for (int r = 0; r < reps; ++r) run();
      hipEventRecord(b);
      hipEventSynchronize(b);
      float ms;
      hipEventElapsedTime(&ms, a, b);
      const double us = ms * 1e3 / reps, moved = kind == 1 ? 2.0 * bytes : 1.0 * bytes;
      printf("%s grid %6d: %8.2f us  %.2f TB/s\n", kind == 0 ? "read      " : kind == 1 ? "read+write" : "write     ", g, us,
             moved / us / 1e6);
    }
  }
  return 0;
}
