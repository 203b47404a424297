// Microbenchmark (design study, round 4): does a scattered gather cost the
// texture path less when it lands in LDS (LDS-DMA: global_load_lds, per-lane
// source address, lane-linear LDS destination) than in VGPRs? fast2d_search
// is bound by the TA/TD path at ~50 TD cycles per scattered gather
// instruction; its gathers are 4-byte (quad) and 16-byte (hex)
// loads from one submap's planes, mostly L2 hits. Each variant: 2048
// workgroups x 4 waves, every wave issues `iters` gather instructions whose
// lanes touch `lines` distinct 128-byte lines (lanes grouped on lines), over a
// 16 MiB buffer; the LDS variants read their slot back (ds_read) and add it.
// Prints cycles per wave-instruction per CU at 2.4 GHz.
//   hipcc --offload-arch=gfx950 -O3 tools/gather_lds_bench.hip -o tools/gather_lds_bench
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>

#define LDS_AS __attribute__((address_space(3)))
#define GLB_AS __attribute__((address_space(1)))

template <int W, bool kLds>
__global__ void __launch_bounds__(256) Gather(const uint32_t* __restrict__ buf, uint32_t mask_lines,
                                              int group, int iters, uint32_t* out) {
  // U gathers in flight per wave between waits (both variants).
  constexpr int U = W == 4 ? 8 : 4;
  __shared__ uint32_t slots[4][U][64 * W / 4];  // one 64 x W slot per gather in flight
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  uint32_t x = (blockIdx.x * 977u + wave * 131u + 1u) * 2654435761u;
  uint32_t acc = 0;
  const uint32_t grp = lane / group, within = lane % group;
  for (int i = 0; i < iters; i += U) {
    const uint32_t* src[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      x = x * 1664525u + 1013904223u;
      const uint32_t line = ((x ^ (grp * 0x9E3779B9u)) * 2246822519u >> 7) & mask_lines;
      src[u] = buf + line * 32 + (within * (W / 4)) % 32;
    }
    if constexpr (kLds) {
#pragma unroll
      for (int u = 0; u < U; ++u) {
        LDS_AS void* dst = (LDS_AS void*)(&slots[wave][u][0]);
        if constexpr (W == 4) __builtin_amdgcn_global_load_lds((GLB_AS void*)src[u], dst, 4, 0, 0);
        else __builtin_amdgcn_global_load_lds((GLB_AS void*)src[u], dst, 16, 0, 0);
      }
      __builtin_amdgcn_s_waitcnt(0x3f70);  // vmcnt(0)
#pragma unroll
      for (int u = 0; u < U; ++u) {
        if constexpr (W == 4) {
          acc += slots[wave][u][lane];
        } else {
          const uint4 v = reinterpret_cast<const uint4*>(&slots[wave][u][0])[lane];
          acc += v.x + v.y + v.z + v.w;
        }
      }
    } else {
      uint4 v[U];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        if constexpr (W == 4) v[u].x = *src[u];
        else v[u] = *reinterpret_cast<const uint4*>(src[u]);
      }
#pragma unroll
      for (int u = 0; u < U; ++u) acc += W == 4 ? v[u].x : v[u].x + v[u].y + v[u].z + v[u].w;
    }
  }
  if (acc == 0x12345678u) out[0] = acc;
}

int main() {
  const uint32_t lines = 1u << 17;  // 16 MiB
  uint32_t *buf, *out;
  (void)hipMalloc(&buf, lines * 128 + 256);
  (void)hipMalloc(&out, 4);
  (void)hipMemset(buf, 1, lines * 128 + 256);
  hipEvent_t a, b;
  (void)hipEventCreate(&a);
  (void)hipEventCreate(&b);
  const int cus = 256, iters = 1000, blocks = 2048, threads = 256;
  auto run = [&](auto kernel, const char* name, int group) {
    hipLaunchKernelGGL(kernel, dim3(blocks), dim3(threads), 0, 0, buf, lines - 1, group, iters, out);
    (void)hipDeviceSynchronize();
    (void)hipEventRecord(a);
    hipLaunchKernelGGL(kernel, dim3(blocks), dim3(threads), 0, 0, buf, lines - 1, group, iters, out);
    (void)hipEventRecord(b);
    (void)hipEventSynchronize(b);
    float ms;
    (void)hipEventElapsedTime(&ms, a, b);
    const double instr = double(blocks) * (threads / 64) * iters;
    std::printf("%-10s lanes/line %2d (%2d lines/instr): %6.1f cycles/instr/CU\n", name, group,
                64 / group, ms * 1e-3 * 2.4e9 * cus / instr);
  };
  for (int g : {1, 4, 16}) {
    run(Gather<4, false>, "vgpr4", g);
    run(Gather<4, true>, "lds4", g);
  }
  for (int g : {1, 4, 8}) {
    run(Gather<16, false>, "vgpr16", g);
    run(Gather<16, true>, "lds16", g);
  }
  return 0;
}
