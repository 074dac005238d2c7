// Workgroup dispatch / residency microbenchmark (gfx950): N workgroups of 256 threads that each
// wait W microseconds (s_memrealtime, 100 MHz) with L bytes of dynamic LDS; reports the kernel span,
// the peak number of workgroups in flight (from per-workgroup start / end stamps) and the rate.
// Build: hipcc --offload-arch=gfx950 -O3 tools/bench_dispatch.hip -o /tmp/bench_dispatch
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>
#include <vector>
#include <algorithm>

__global__ __launch_bounds__(256) void spin(uint64_t* stamps, int wait_ticks, int touch_lds) {
    extern __shared__ float sm[];
    const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
    if (touch_lds) sm[threadIdx.x] = (float)threadIdx.x;
    uint64_t t = t0;
    while (t - t0 < (uint64_t)wait_ticks) {
        __builtin_amdgcn_s_sleep(2);
        t = __builtin_amdgcn_s_memrealtime();
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        stamps[2 * blockIdx.x] = t0;
        stamps[2 * blockIdx.x + 1] = __builtin_amdgcn_s_memrealtime() + (touch_lds ? (uint64_t)sm[5] * 0 : 0);
    }
}

int main(int argc, char** argv) {
    uint64_t* d;
    const int NMAX = 8192;
    hipMalloc(&d, sizeof(uint64_t) * 2 * NMAX);
    std::vector<uint64_t> h(2 * NMAX);
    printf("%6s %6s %8s  %9s %9s %9s %9s\n", "blocks", "wait", "lds", "span_us", "inflight", "WG/us", "fill_us");
    const bool sweep = argc > 1;
    std::vector<int> ldss = sweep ? std::vector<int>{26624, 27648, 28672, 29696, 30720, 31744, 32512, 32768, 53248, 54272}
                                  : std::vector<int>{0, 32768, 65536};
    std::vector<int> waits = sweep ? std::vector<int>{5} : std::vector<int>{1, 5, 12};
    std::vector<int> ns = sweep ? std::vector<int>{4608} : std::vector<int>{512, 2304, 4608};
    for (int lds : ldss) {
        for (int wait_us : waits) {
            for (int n : ns) {
                for (int rep = 0; rep < 2; ++rep)
                    hipLaunchKernelGGL(spin, dim3(n), dim3(256), lds, 0, d, wait_us * 100, lds > 0);
                if (lds > 65536) (void)hipFuncSetAttribute((const void*)spin, hipFuncAttributeMaxDynamicSharedMemorySize, lds);
                hipDeviceSynchronize();
                hipMemcpy(h.data(), d, sizeof(uint64_t) * 2 * n, hipMemcpyDeviceToHost);
                uint64_t lo = UINT64_MAX, hi = 0;
                std::vector<std::pair<uint64_t, int>> ev;
                for (int i = 0; i < n; ++i) {
                    lo = std::min(lo, h[2 * i]);
                    hi = std::max(hi, h[2 * i + 1]);
                    ev.push_back({h[2 * i], +1});
                    ev.push_back({h[2 * i + 1], -1});
                }
                std::sort(ev.begin(), ev.end());
                int cur = 0, peak = 0;
                for (auto& e : ev) { cur += e.second; peak = std::max(peak, cur); }
                // time until the first `peak` workgroups had started
                std::vector<uint64_t> starts(n);
                for (int i = 0; i < n; ++i) starts[i] = h[2 * i];
                std::sort(starts.begin(), starts.end());
                const double fill = (starts[std::min(peak, n) - 1] - lo) / 100.0;
                const double span = (hi - lo) / 100.0;
                printf("%6d %6d %8d  %9.2f %9d %9.1f %9.2f\n", n, wait_us, lds, span, peak, n / span, fill);
            }
        }
    }
    return 0;
}
