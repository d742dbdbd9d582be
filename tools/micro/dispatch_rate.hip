// Dispatch-rate probe: N empty kernels per stream on S streams, queued behind a ~spin kernel so the
// host enqueue (one thread, ~2.8 us a launch) is done before they run; GPU time from events after
// the spin to after the last kernel, max over streams. Tells whether back-to-back short kernels
// are bound by the command processor's dispatch rate.   ./dispatch_rate [kernels per stream] [max streams]
#include <hip/hip_runtime.h>
#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <vector>

__global__ void k_empty(int* p) { if (p && threadIdx.x == 1024) p[0] = 1; }
__global__ void k_spin(long long cycles) {
    const long long t0 = clock64();
    while (clock64() - t0 < cycles) __builtin_amdgcn_s_sleep(10);
}

int main(int argc, char** argv) {
    const int n = argc > 1 ? atoi(argv[1]) : 1000;
    const int smax = argc > 2 ? atoi(argv[2]) : 8;
    std::vector<hipStream_t> st(smax);
    std::vector<hipEvent_t> e0(smax), e1(smax);
    for (int s = 0; s < smax; s++) {
        (void)hipStreamCreateWithFlags(&st[s], hipStreamNonBlocking);
        (void)hipEventCreate(&e0[s]);
        (void)hipEventCreate(&e1[s]);
    }
    for (int grid : {1, 256}) {
        for (int S = 1; S <= smax; S *= 2) {
            for (int rep = 0; rep < 2; rep++) {
                (void)hipDeviceSynchronize();
                for (int s = 0; s < S; s++) {
                    hipLaunchKernelGGL(k_spin, dim3(1), dim3(64), 0, st[s], 400000000LL);   // long enough to cover the enqueue
                    (void)hipEventRecord(e0[s], st[s]);
                }
                for (int i = 0; i < n; i++)
                    for (int s = 0; s < S; s++) hipLaunchKernelGGL(k_empty, dim3(grid), dim3(64), 0, st[s], nullptr);
                for (int s = 0; s < S; s++) (void)hipEventRecord(e1[s], st[s]);
                (void)hipDeviceSynchronize();
                float mx = 0, mn = 1e30f;
                for (int s = 0; s < S; s++) {
                    float ms = 0;
                    (void)hipEventElapsedTime(&ms, e0[s], e1[s]);
                    mx = std::max(mx, ms);
                    mn = std::min(mn, ms);
                }
                if (rep == 1)
                    printf("grid %4d streams %d: %5d kernels per stream, GPU %.2f-%.2f us per kernel per stream, %.2f us per kernel overall\n",
                           grid, S, n, 1e3 * mn / n, 1e3 * mx / n, 1e3 * mx / (n * S));
            }
        }
    }
    return 0;
}
