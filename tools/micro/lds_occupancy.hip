// How many one-wave workgroups of a given LDS size are resident per CU at
// once (not part of the product; sizes the trace kernel's LDS).  Each
// workgroup spins ~200 us; the ones that started before the first of them
// ended were resident together.
//   hipcc --offload-arch=gfx950 -O2 lds_occupancy.hip -o lds_occ && ./lds_occ
#include <hip/hip_runtime.h>
#include <algorithm>
#include <cstdio>
#include <vector>

__global__ __launch_bounds__(64) void spin(unsigned long long* t0, unsigned long long ticks) {
  extern __shared__ float4 sm[];
  sm[threadIdx.x] = make_float4(1.f, 2.f, 3.f, 4.f);
  __syncthreads();
  const unsigned long long s = wall_clock64();
  while (wall_clock64() - s < ticks) {
  }
  if (threadIdx.x == 0) t0[blockIdx.x] = s + (unsigned long long)sm[threadIdx.x + 1].x;
}

int main() {
  hipDeviceProp_t p;
  if (hipGetDeviceProperties(&p, 0) != hipSuccess) return 1;
  const int cus = p.multiProcessorCount, G = cus * 40;
  unsigned long long* d = nullptr;
  if (hipMalloc(&d, G * sizeof(unsigned long long)) != hipSuccess) return 1;
  for (int lds : {4096, 6656, 6784, 7168, 7680, 7808, 8192}) {
    int occ = 0;
    (void)hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, spin, 64, lds);
    hipLaunchKernelGGL(spin, dim3(G), dim3(64), lds, 0, d, 20000ull);  // 200 us at 100 MHz
    if (hipDeviceSynchronize() != hipSuccess) return 1;
    std::vector<unsigned long long> h(G);
    (void)hipMemcpy(h.data(), d, G * sizeof(unsigned long long), hipMemcpyDeviceToHost);
    for (auto& x : h) x -= 1;  // the LDS value added above (1.0f -> 1)
    const unsigned long long first = *std::min_element(h.begin(), h.end());
    int together = 0;
    for (auto x : h) together += x < first + 10000ull;  // started in the first 100 us
    printf("{\"lds\": %d, \"api_blocks_per_cu\": %d, \"resident_per_cu\": %.2f}\n", lds, occ, (double)together / cus);
  }
  (void)hipFree(d);
  return 0;
}
