// Round-trip latency of a device scalar read: kernel -> D2H copy -> host sees it -> next kernel.
#include <hip/hip_runtime.h>
#include <chrono>
#include <cstdio>
#include <cstring>
#include <immintrin.h>
__global__ void k_bump(unsigned long long *x) { if (threadIdx.x == 0) x[0] += 1; }
#define H(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("err %s line %d\n", hipGetErrorString(e), __LINE__); return 1; } } while (0)
int main() {
    hipStream_t st; H(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
    unsigned long long *d; H(hipMalloc(&d, 64)); H(hipMemset(d, 0, 64));
    unsigned long long *pin; H(hipHostMalloc(&pin, 64, hipHostMallocDefault));
    hipEvent_t ev; H(hipEventCreateWithFlags(&ev, hipEventDisableTiming));
    const int R = 2000;
    for (int mode = 0; mode < 5; mode++) {
        auto t0 = std::chrono::steady_clock::now();
        unsigned long long v = 0;
        for (int i = 0; i < R; i++) {
            k_bump<<<1, 64, 0, st>>>(d);
            if (mode == 0) { H(hipMemcpyAsync(&v, d, 8, hipMemcpyDeviceToHost, st)); H(hipStreamSynchronize(st)); }
            else if (mode == 1) { H(hipMemcpyAsync(pin, d, 8, hipMemcpyDeviceToHost, st)); H(hipStreamSynchronize(st)); v = *pin; }
            else if (mode == 2) { H(hipMemcpyAsync(pin, d, 8, hipMemcpyDeviceToHost, st)); H(hipEventRecord(ev, st));
                while (hipEventQuery(ev) == hipErrorNotReady) _mm_pause(); v = *pin; }
            else if (mode == 3) { H(hipMemcpyAsync(&v, d, 8, hipMemcpyDeviceToHost, st)); H(hipEventRecord(ev, st));
                while (hipEventQuery(ev) == hipErrorNotReady) _mm_pause(); }
            else { H(hipStreamSynchronize(st)); }
        }
        auto t1 = std::chrono::steady_clock::now();
        printf("mode %d (%s): %.1f us per round trip (v=%llu)\n", mode,
               mode == 0 ? "pageable copy + stream sync" : mode == 1 ? "pinned copy + stream sync" :
               mode == 2 ? "pinned copy + event spin" : mode == 3 ? "pageable copy + event spin" : "kernel + stream sync only",
               std::chrono::duration<double, std::micro>(t1 - t0).count() / R, v);
    }
    return 0;
}
