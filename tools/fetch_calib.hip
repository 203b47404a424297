// FETCH_SIZE calibration for the access patterns of fast2d_search (round 4).
//
// The guide calibrates rocprofv3's FETCH_SIZE only for wide coalesced
// streaming reads (it reports half of the bytes there). fast2d_search issues
// scattered 4-byte (quad) and 16-byte (hex) gathers, so this program reads
// KNOWN byte counts from cold HBM with those patterns, one dispatch each, and
// prints for every dispatch the distinct 32 / 64 / 128-byte units it touched
// (computed on the host from the same hash). tools/fetch_calib.py joins that
// with a `rocprofv3 --pmc FETCH_SIZE` pass over this program to give FETCH's
// factor per pattern.
//
// Every measured dispatch is preceded by a 1 GiB streaming read of another
// buffer, so the Infinity Cache (256 MiB) and the L2s hold none of the data
// read next; the scatter targets span 8 GiB.
//   hipcc --offload-arch=gfx950 -O3 tools/fetch_calib.hip -o tools/fetch_calib
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>
#include <cstdio>
#include <vector>

__host__ __device__ inline uint64_t Mix(uint64_t x) {  // splitmix64
  x += 0x9E3779B97F4A7C15ull;
  x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
  x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
  return x ^ (x >> 31);
}

// Lane t reads `width` bytes (4 or 16) at a random aligned offset; `group`
// consecutive lanes share a random 128-byte line and read consecutive items
// of it (group = 1: every lane its own line).
template <int W>
__global__ void Scatter(const uint8_t* __restrict__ buf, uint64_t lines, int group, uint64_t n,
                        uint32_t* out) {
  const uint64_t t = blockIdx.x * static_cast<uint64_t>(blockDim.x) + threadIdx.x;
  if (t >= n) return;
  const uint64_t g = t / group, k = t % group;
  const uint64_t line = Mix(g * 0x2545F4914F6CDD1Dull + 17) % lines;
  const uint64_t off = line * 128 + (k * W) % 128;
  uint32_t v;
  if (W == 4) {
    v = *reinterpret_cast<const uint32_t*>(buf + off);
  } else {
    const uint4 q = *reinterpret_cast<const uint4*>(buf + off);
    v = q.x + q.y + q.z + q.w;
  }
  if (v == 0x9E3779B9u) out[0] = v;  // keeps the load
}

__global__ void Stream(const uint4* __restrict__ buf, uint64_t n16, uint32_t* out) {
  uint32_t acc = 0;
  for (uint64_t i = blockIdx.x * static_cast<uint64_t>(blockDim.x) + threadIdx.x; i < n16;
       i += static_cast<uint64_t>(gridDim.x) * blockDim.x) {
    const uint4 q = buf[i];
    acc += q.x ^ q.y ^ q.z ^ q.w;
  }
  if (acc == 0x9E3779B9u) out[0] = acc;
}

struct Case {
  const char* name;
  int width, group;
  uint64_t n;
};

int main() {
  const uint64_t kScatterBytes = 8ull << 30, kFlushBytes = 1ull << 30, kStreamBytes = 1ull << 30;
  uint8_t *scatter = nullptr, *flush = nullptr, *stream = nullptr;
  uint32_t* out = nullptr;
  if (hipMalloc(&scatter, kScatterBytes) != hipSuccess || hipMalloc(&flush, kFlushBytes) != hipSuccess ||
      hipMalloc(&stream, kStreamBytes) != hipSuccess || hipMalloc(&out, 4) != hipSuccess) {
    std::fprintf(stderr, "allocation failed\n");
    return 1;
  }
  (void)hipMemset(scatter, 1, kScatterBytes);
  (void)hipMemset(flush, 2, kFlushBytes);
  (void)hipMemset(stream, 3, kStreamBytes);
  const uint64_t lines = kScatterBytes / 128;
  auto flush_caches = [&] {
    hipLaunchKernelGGL(Stream, dim3(4096), dim3(256), 0, 0, reinterpret_cast<const uint4*>(flush),
                       kFlushBytes / 16, out);
  };
  // Distinct 32 / 64 / 128-byte units a case touches (host replay of the hash).
  auto distinct = [&](const Case& c, uint64_t unit) {
    std::vector<uint64_t> u;
    u.reserve(c.n);
    for (uint64_t t = 0; t < c.n; ++t) {
      const uint64_t g = t / c.group, k = t % c.group;
      const uint64_t line = Mix(g * 0x2545F4914F6CDD1Dull + 17) % lines;
      const uint64_t off = line * 128 + (k * c.width) % 128;
      u.push_back(off / unit);
    }
    std::sort(u.begin(), u.end());
    return static_cast<uint64_t>(std::unique(u.begin(), u.end()) - u.begin());
  };
  std::printf("{\"dispatches\": [\n");
  // Dispatch order (what rocprofv3 sees): flush, stream 1 GiB, then per case
  // flush + scatter.
  flush_caches();
  hipLaunchKernelGGL(Stream, dim3(4096), dim3(256), 0, 0, reinterpret_cast<const uint4*>(stream),
                     kStreamBytes / 16, out);
  (void)hipDeviceSynchronize();
  std::printf("  {\"name\": \"stream16\", \"index\": 1, \"bytes_read\": %llu, \"u32\": %llu, "
              "\"u64\": %llu, \"u128\": %llu},\n",
              (unsigned long long)kStreamBytes, (unsigned long long)(kStreamBytes / 32),
              (unsigned long long)(kStreamBytes / 64), (unsigned long long)(kStreamBytes / 128));
  const Case cases[] = {{"scatter4", 4, 1, 1ull << 24},     {"scatter16", 16, 1, 1ull << 24},
                        {"scatter4_x4", 4, 4, 1ull << 26},  {"scatter16_x4", 16, 4, 1ull << 25},
                        {"scatter4_x16", 4, 16, 1ull << 26}, {"scatter16_x8", 16, 8, 1ull << 25}};
  int index = 2;
  for (size_t i = 0; i < sizeof(cases) / sizeof(cases[0]); ++i) {
    const Case& c = cases[i];
    flush_caches();
    ++index;
    const dim3 grid(static_cast<uint32_t>((c.n + 255) / 256));
    if (c.width == 4)
      hipLaunchKernelGGL(Scatter<4>, grid, dim3(256), 0, 0, scatter, lines, c.group, c.n, out);
    else
      hipLaunchKernelGGL(Scatter<16>, grid, dim3(256), 0, 0, scatter, lines, c.group, c.n, out);
    (void)hipDeviceSynchronize();
    std::printf("  {\"name\": \"%s\", \"index\": %d, \"bytes_read\": %llu, \"u32\": %llu, "
                "\"u64\": %llu, \"u128\": %llu}%s\n",
                c.name, index, (unsigned long long)(c.n * c.width),
                (unsigned long long)distinct(c, 32), (unsigned long long)distinct(c, 64),
                (unsigned long long)distinct(c, 128), i + 1 < sizeof(cases) / sizeof(cases[0]) ? "," : "");
    ++index;
  }
  std::printf("]}\n");
  return 0;
}
