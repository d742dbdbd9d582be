// PCIe duplex probe: HBM <-> pinned host copies by the SDMA engines (hipMemcpyAsync) and by kernels
// that read / write the host pages through their device address (zero-copy), alone and two at once on
// two streams. Tells whether an H2D and a D2H can share the link at full duplex, and by which path.
//   ./link_duplex [MiB]
#include <hip/hip_runtime.h>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <functional>

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

// grid-stride 16-byte copy (n a multiple of 16)
__global__ void k_copy(u32x4* __restrict__ d, const u32x4* __restrict__ s, size_t n16) {
    for (size_t i = blockIdx.x * size_t(blockDim.x) + threadIdx.x; i < n16; i += size_t(gridDim.x) * blockDim.x)
        d[i] = __builtin_nontemporal_load(s + i);
}

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e_)); exit(1); } } while (0)

int main(int argc, char** argv) {
    const size_t n = size_t(argc > 1 ? atoi(argv[1]) : 512) << 20;
    void *da, *db, *ha, *hb, *hda, *hdb;
    CK(hipMalloc(&da, n)); CK(hipMalloc(&db, n));
    CK(hipHostMalloc(&ha, n, hipHostMallocDefault)); CK(hipHostMalloc(&hb, n, hipHostMallocDefault));
    CK(hipHostGetDevicePointer(&hda, ha, 0)); CK(hipHostGetDevicePointer(&hdb, hb, 0));
    CK(hipMemset(da, 1, n)); CK(hipMemset(db, 2, n));
    hipStream_t s1, s2;
    CK(hipStreamCreateWithFlags(&s1, hipStreamNonBlocking)); CK(hipStreamCreateWithFlags(&s2, hipStreamNonBlocking));
    const size_t n16 = n / 16;
    auto h2d_sdma = [&](hipStream_t s) { CK(hipMemcpyAsync(da, ha, n, hipMemcpyHostToDevice, s)); };
    auto d2h_sdma = [&](hipStream_t s) { CK(hipMemcpyAsync(hb, db, n, hipMemcpyDeviceToHost, s)); };
    auto grid = [](int g) { return dim3(g); };
    int G = argc > 2 ? atoi(argv[2]) : 1024;
    auto h2d_kern = [&](hipStream_t s) { hipLaunchKernelGGL(k_copy, grid(G), dim3(256), 0, s, (u32x4*)da, (const u32x4*)hda, n16); };
    auto d2h_kern = [&](hipStream_t s) { hipLaunchKernelGGL(k_copy, grid(G), dim3(256), 0, s, (u32x4*)hdb, (const u32x4*)db, n16); };
    auto timed = [&](std::function<void()> f) {
        double best = 1e9;
        for (int r = 0; r < 5; r++) {
            CK(hipDeviceSynchronize());
            auto t0 = std::chrono::steady_clock::now();
            f();
            CK(hipDeviceSynchronize());
            best = std::min(best, std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count());
        }
        return best;
    };
    printf("bytes %zu, kernel grid %d x 256\n", n, G);
    printf("h2d sdma   %6.2f GB/s\n", n / timed([&] { h2d_sdma(s1); }) / 1e9);
    printf("d2h sdma   %6.2f GB/s\n", n / timed([&] { d2h_sdma(s2); }) / 1e9);
    printf("h2d kernel %6.2f GB/s\n", n / timed([&] { h2d_kern(s1); }) / 1e9);
    printf("d2h kernel %6.2f GB/s\n", n / timed([&] { d2h_kern(s2); }) / 1e9);
    double t;
    t = timed([&] { h2d_sdma(s1); d2h_sdma(s2); });   printf("both sdma              %6.2f GB/s total\n", 2 * n / t / 1e9);
    t = timed([&] { h2d_sdma(s1); d2h_kern(s2); });   printf("h2d sdma + d2h kernel  %6.2f GB/s total\n", 2 * n / t / 1e9);
    t = timed([&] { h2d_kern(s1); d2h_sdma(s2); });   printf("h2d kernel + d2h sdma  %6.2f GB/s total\n", 2 * n / t / 1e9);
    t = timed([&] { h2d_kern(s1); d2h_kern(s2); });   printf("both kernel            %6.2f GB/s total\n", 2 * n / t / 1e9);
    return 0;
}
