// Waves per CU admitted for workgroups of W waves with a given static LDS
// size per wave: the runtime's occupancy query, and the measured peak of
// concurrently resident waves (each wave spins ~60 us on the 100 MHz
// constant clock and records its start and end; the peak overlap / the CU
// count). What caps the parse kernel's residency (one-wave workgroups,
// 8,960 B of LDS each).
//   lds_occ
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <algorithm>
#include <vector>

template <int B, int W>
__global__ void __launch_bounds__(64 * W) k(uint64_t* out, uint64_t ticks) {
    __shared__ int s[B > 0 ? W * B / 4 : 1];
    const int t = threadIdx.x;
    if (B > 0) s[t] = t;
    __syncthreads();
    const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
    while (__builtin_amdgcn_s_memrealtime() - t0 < ticks) {
    }
    const uint64_t t1 = __builtin_amdgcn_s_memrealtime();
    if ((t & 63) == 0) {
        const uint64_t w = (uint64_t)blockIdx.x * W + (t >> 6);
        out[2 * w] = t0;
        out[2 * w + 1] = t1 + (B > 0 && s[(t + 1) % (W * 64)] == 12345);
    }
}

template <int B, int W>
static void probe(uint64_t* d, int cus) {
    const int nw = cus * 40, nb = nw / W;
    int blocks = 0;
    (void)hipOccupancyMaxActiveBlocksPerMultiprocessor(&blocks, k<B, W>, 64 * W, 0);
    hipLaunchKernelGGL((k<B, W>), dim3(nb), dim3(64 * W), 0, 0, d, (uint64_t)6000);   // 60 us
    if (hipDeviceSynchronize() != hipSuccess) { printf("launch failed\n"); return; }
    std::vector<uint64_t> h(2 * nw);
    (void)hipMemcpy(h.data(), d, 16ull * nw, hipMemcpyDeviceToHost);
    std::vector<std::pair<uint64_t, int>> ev;
    for (int i = 0; i < nw; ++i) { ev.push_back({h[2 * i], 1}); ev.push_back({h[2 * i + 1], -1}); }
    std::sort(ev.begin(), ev.end(), [](auto a, auto b) { return a.first < b.first || (a.first == b.first && a.second < b.second); });
    int cur = 0, peak = 0;
    for (auto& e : ev) { cur += e.second; peak = std::max(peak, cur); }
    printf("%d-wave workgroups, %6d B of LDS per wave: occupancy query %2d waves/CU, measured peak %.2f waves per CU\n",
           W, B, blocks * W, (double)peak / cus);
}

int main() {
    int cus = 0;
    (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
    uint64_t* d = nullptr;
    if (hipMalloc(&d, 16ull * cus * 40) != hipSuccess) return 1;
    probe<0, 1>(d, cus); probe<4096, 1>(d, cus); probe<7168, 1>(d, cus); probe<7680, 1>(d, cus);
    probe<7936, 1>(d, cus); probe<8064, 1>(d, cus); probe<8192, 1>(d, cus); probe<8960, 1>(d, cus);
    probe<9216, 1>(d, cus);
    probe<0, 2>(d, cus); probe<8192, 2>(d, cus); probe<8960, 2>(d, cus);
    probe<8192, 4>(d, cus); probe<8960, 4>(d, cus);
    return 0;
}
