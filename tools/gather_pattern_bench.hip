// Microbenchmark (design study, round 4): what a scattered gather costs the
// texture path as a function of how its 64 lanes fall on 128-byte lines.
// fast2d_search's gathers touch 10-14 lines per instruction yet cost ~50 TD
// cycles, more than the ~2.2 cycles per distinct line a
// uniform pattern costs; this separates the candidate factors:
//   * distinct lines per instruction (64 / G lanes per line),
//   * whether a line's lanes are adjacent (line = lane / G: every 4-lane
//     group on one line) or strided (line = lane % (64 / G): every 4-lane
//     group on 4 lines),
//   * load width (dword or dwordx4),
//   * working set: 2 MiB (L2-resident on every XCD) or 64 MiB (past L2).
// Every wave issues `iters` gathers, U in flight; prints cycles per
// wave-instruction per CU at 2.4 GHz.
//   hipcc --offload-arch=gfx950 -O3 tools/gather_pattern_bench.hip -o tools/gather_pattern_bench
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>

template <int W, bool kStrided>
__global__ void __launch_bounds__(256) Gather(const uint32_t* __restrict__ buf, uint32_t mask_lines,
                                              int group, int iters, uint32_t* out) {
  constexpr int U = 8;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  uint32_t x = (blockIdx.x * 977u + wave * 131u + 1u) * 2654435761u;
  uint32_t acc = 0;
  const int nlines = 64 / group;
  const uint32_t grp = kStrided ? lane % nlines : lane / group;
  const uint32_t within = kStrided ? lane / nlines : lane % group;
  for (int i = 0; i < iters; i += U) {
    uint4 v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      x = x * 1664525u + 1013904223u;
      const uint32_t line = ((x ^ (grp * 0x9E3779B9u)) * 2246822519u >> 7) & mask_lines;
      const uint32_t* src = buf + line * 32 + (within * (W / 4)) % 32;
      if constexpr (W == 4) v[u].x = *src;
      else v[u] = *reinterpret_cast<const uint4*>(src);
    }
#pragma unroll
    for (int u = 0; u < U; ++u) acc += W == 4 ? v[u].x : v[u].x + v[u].y + v[u].z + v[u].w;
  }
  if (acc == 0x12345678u) out[0] = acc;
}

int main() {
  const uint32_t max_lines = 1u << 19;  // 64 MiB
  uint32_t *buf, *out;
  (void)hipMalloc(&buf, max_lines * 128 + 256);
  (void)hipMalloc(&out, 4);
  (void)hipMemset(buf, 1, max_lines * 128 + 256);
  hipEvent_t a, b;
  (void)hipEventCreate(&a);
  (void)hipEventCreate(&b);
  const int cus = 256, iters = 512, blocks = 4096, threads = 256;
  auto run = [&](auto kernel, const char* name, int group, uint32_t lines) {
    hipLaunchKernelGGL(kernel, dim3(blocks), dim3(threads), 0, 0, buf, lines - 1, group, iters, out);
    (void)hipDeviceSynchronize();
    (void)hipEventRecord(a);
    hipLaunchKernelGGL(kernel, dim3(blocks), dim3(threads), 0, 0, buf, lines - 1, group, iters, out);
    (void)hipEventRecord(b);
    (void)hipEventSynchronize(b);
    float ms;
    (void)hipEventElapsedTime(&ms, a, b);
    const double instr = double(blocks) * (threads / 64) * iters;
    std::printf("%-12s set %5u KiB  lanes/line %2d (%2d lines/instr): %6.1f cycles/instr/CU\n", name,
                lines / 8, group, 64 / group, ms * 1e-3 * 2.4e9 * cus / instr);
  };
  for (uint32_t lines : {1u << 14, max_lines}) {  // 2 MiB, 64 MiB
    for (int g : {1, 2, 4, 8, 16}) {
      run(Gather<4, false>, "b32 adjacent", g, lines);
      if (g > 1) run(Gather<4, true>, "b32 strided", g, lines);
    }
    for (int g : {1, 2, 4, 8}) {
      run(Gather<16, false>, "b128 adjacent", g, lines);
      if (g > 1) run(Gather<16, true>, "b128 strided", g, lines);
    }
  }
  return 0;
}
