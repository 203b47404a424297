// Microbenchmark: cost of one wave-wide gather instruction on gfx950 by width
// (dword / dwordx2 / dwordx4) and by address spread (lines per instruction),
// buffer resident in L2/MALL. Prints ns per wave-instruction per CU.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <cstdlib>

template <int W>
__global__ void gather(const uint32_t* __restrict__ buf, uint32_t mask_words, int spread, int iters,
                       uint32_t* out) {
  const int lane = threadIdx.x & 63;
  uint32_t x = (blockIdx.x * 977u + (threadIdx.x >> 6) * 131u) * 2654435761u;
  uint32_t acc = 0;
  const __amdgpu_buffer_rsrc_t rs =
      __builtin_amdgcn_make_buffer_rsrc(const_cast<uint32_t*>(buf), 0, (mask_words + 64) * 4, 0x00020000);
  for (int i = 0; i < iters; ++i) {
    x = x * 1664525u + 1013904223u;  // wave-uniform base
    // spread: lanes fall into `spread` groups; a group's lanes read consecutive
    // W-dword items of one region, groups far apart.
    const uint32_t grp = lane % spread;
    const uint32_t within = lane / spread;
    const uint32_t base = ((x ^ (grp * 0x9E3779B9u)) & mask_words) & ~63u;
    const uint32_t off = (base + within * W) * 4;
    if (W == 1) acc += __builtin_amdgcn_raw_buffer_load_b32(rs, off, 0, 0);
    if (W == 2) { auto v = __builtin_amdgcn_raw_buffer_load_b64(rs, off, 0, 0); acc += v[0] + v[1]; }
    if (W == 4) { auto v = __builtin_amdgcn_raw_buffer_load_b128(rs, off, 0, 0); acc += v[0] + v[1] + v[2] + v[3]; }
  }
  if (acc == 0x12345678u) out[0] = acc;
}

int main(int argc, char** argv) {
  const uint32_t words = 1u << (argc > 1 ? atoi(argv[1]) : 22);  // 2^k words
  uint32_t* buf; uint32_t* out;
  hipMalloc(&buf, (words + 64) * 4); hipMalloc(&out, 4);
  hipMemset(buf, 1, (words + 64) * 4);
  hipEvent_t a, b; hipEventCreate(&a); hipEventCreate(&b);
  int cus = 256;
  const int iters = 2000, blocks = cus * 8, threads = 256;
  printf("buffer %u KB\n", words / 256);
  for (int spread : {1, 4, 16, 32, 64}) {
    for (int w : {1, 4}) {
      auto launch = [&]() {
        if (w == 1) hipLaunchKernelGGL(gather<1>, dim3(blocks), dim3(threads), 0, 0, buf, words - 1, spread, iters, out);
        if (w == 2) hipLaunchKernelGGL(gather<2>, dim3(blocks), dim3(threads), 0, 0, buf, words - 1, spread, iters, out);
        if (w == 4) hipLaunchKernelGGL(gather<4>, dim3(blocks), dim3(threads), 0, 0, buf, words - 1, spread, iters, out);
      };
      launch(); hipDeviceSynchronize();
      hipEventRecord(a); launch(); hipEventRecord(b); hipEventSynchronize(b);
      float ms; hipEventElapsedTime(&ms, a, b);
      const double instr = double(blocks) * (threads / 64) * iters;
      printf("spread %2d width %d: %.3f ms, %.2f cycles/instr/CU (at 2.4 GHz)\n", spread, w, ms,
             ms * 1e-3 * 2.4e9 * cus / instr);
    }
  }
  return 0;
}
