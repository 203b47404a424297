// Microbenchmark (design study): cost of one wave-wide buffer gather on gfx950
// when lanes form contiguous blocks (lanes [b*blk, (b+1)*blk) read consecutive
// items of one random region, blocks far apart), and when every lane re-reads
// the line it read `reuse` instructions earlier (L1-resident). Buffer in L2.
// Prints cycles per wave-instruction per CU at 2.4 GHz.
//   hipcc --offload-arch=gfx950 -O3 tools/gather_bench2.hip -o gather_bench2
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

template <int W>
__global__ void gather(const uint32_t* __restrict__ buf, uint32_t mask_words, int blk, int reuse,
                       int iters, uint32_t* out) {
  const int lane = threadIdx.x & 63;
  uint32_t x = (blockIdx.x * 977u + (threadIdx.x >> 6) * 131u) * 2654435761u;
  uint32_t acc = 0;
  const __amdgpu_buffer_rsrc_t rs =
      __builtin_amdgcn_make_buffer_rsrc(const_cast<uint32_t*>(buf), 0, (mask_words + 256) * 4, 0x00020000);
  const uint32_t grp = lane / blk, within = lane % blk;
  uint32_t base = 0;
  for (int i = 0; i < iters; ++i) {
    // A new random region every `reuse` instructions; in between the lanes
    // re-read the same items (L1 hits after the first).
    if (reuse <= 1 || i % reuse == 0) {
      x = x * 1664525u + 1013904223u;
      base = ((x ^ (grp * 0x9E3779B9u)) & mask_words) & ~63u;
    }
    const uint32_t off = (base + within * W) * 4;
    if (W == 1) acc += __builtin_amdgcn_raw_buffer_load_b32(rs, off, 0, 0);
    if (W == 4) { auto v = __builtin_amdgcn_raw_buffer_load_b128(rs, off, 0, 0); acc += v[0] + v[1] + v[2] + v[3]; }
  }
  if (acc == 0x12345678u) out[0] = acc;
}

int main() {
  const uint32_t words = 1u << 20;  // 4 MB
  uint32_t* buf; uint32_t* out;
  hipMalloc(&buf, (words + 256) * 4); hipMalloc(&out, 4);
  hipMemset(buf, 1, (words + 256) * 4);
  hipEvent_t a, b; hipEventCreate(&a); hipEventCreate(&b);
  const int cus = 256, iters = 2000, blocks = cus * 8, threads = 256;
  auto run = [&](int w, int blk, int reuse) {
    auto launch = [&]() {
      if (w == 1) hipLaunchKernelGGL(gather<1>, dim3(blocks), dim3(threads), 0, 0, buf, words - 1, blk, reuse, iters, out);
      else hipLaunchKernelGGL(gather<4>, dim3(blocks), dim3(threads), 0, 0, buf, words - 1, blk, reuse, iters, out);
    };
    launch(); hipDeviceSynchronize();
    hipEventRecord(a); launch(); hipEventRecord(b); hipEventSynchronize(b);
    float ms; hipEventElapsedTime(&ms, a, b);
    const double instr = double(blocks) * (threads / 64) * iters;
    printf("width %d block %2d reuse %d: %.2f cycles/instr/CU\n", w, blk, reuse,
           ms * 1e-3 * 2.4e9 * cus / instr);
  };
  for (int blk : {1, 2, 4, 8, 16, 64}) run(4, blk, 1);
  for (int blk : {1, 4, 8, 32, 64}) run(1, blk, 1);
  for (int reuse : {2, 4, 8}) run(4, 1, reuse);
  for (int reuse : {2, 4, 8}) run(1, 1, reuse);
  return 0;
}
