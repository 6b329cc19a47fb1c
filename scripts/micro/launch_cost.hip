// Host cost of one kernel launch with a MatchArgs-sized (512 B) argument, and the decision -> kernel-start
// latency, for the launch forms the front end could use (diagnostics for DESIGN §8):
//   A. triple-chevron                      B. hipExtLaunchKernelGGL, null events (what lio_match does)
//   C. hipModuleLaunchKernel on a hipFunction_t cached by hipGetFuncBySymbol (kernelParams)
//   D. as C with the argument buffer passed through `extra` (HIP_LAUNCH_PARAM_BUFFER_POINTER)
// Each: median host microseconds per launch call (1000 back-to-back launches of a 1-block kernel, the
// queue drained between batches of 100), then a round trip: launch -> kernel writes a host-mapped
// flag -> host sees it.
#include <hip/hip_ext.h>
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <vector>

struct Big {
    unsigned long long* flag;
    unsigned long long seq;
    float pad[124];
};

typedef __attribute__((address_space(1))) unsigned long long gull;

__global__ void k_big(Big a) {
    if (threadIdx.x == 0 && a.flag) __hip_atomic_store((gull*)a.flag, a.seq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

using clk = std::chrono::steady_clock;
static double us(clk::time_point a, clk::time_point b) { return std::chrono::duration<double, std::micro>(b - a).count(); }
static double median(std::vector<double> v) {
    std::sort(v.begin(), v.end());
    return v[v.size() / 2];
}

int main() {
    hipStream_t st;
    (void)hipStreamCreateWithFlags(&st, hipStreamNonBlocking);
    unsigned long long *h, *d;
    (void)hipHostMalloc(&h, 64, hipHostMallocMapped | hipHostMallocCoherent);
    (void)hipHostGetDevicePointer((void**)&d, h, 0);
    volatile unsigned long long* hv = h;
    *hv = 0;
    hipFunction_t f = nullptr;
    if (hipGetFuncBySymbol(&f, reinterpret_cast<const void*>(&k_big)) != hipSuccess) {
        std::printf("hipGetFuncBySymbol failed\n");
        return 1;
    }
    Big a{};
    a.flag = nullptr;
    auto launch = [&](int form) {
        switch (form) {
        case 0: k_big<<<1, 64, 0, st>>>(a); break;
        case 1: hipExtLaunchKernelGGL(k_big, dim3(1), dim3(64), 0, st, nullptr, nullptr, 0, a); break;
        case 2: {
            void* params[] = {&a};
            (void)hipModuleLaunchKernel(f, 1, 1, 1, 64, 1, 1, 0, st, params, nullptr);
            break;
        }
        default: {
            size_t sz = sizeof(a);
            void* extra[] = {HIP_LAUNCH_PARAM_BUFFER_POINTER, &a, HIP_LAUNCH_PARAM_BUFFER_SIZE, &sz, HIP_LAUNCH_PARAM_END};
            (void)hipModuleLaunchKernel(f, 1, 1, 1, 64, 1, 1, 0, st, nullptr, extra);
        }
        }
    };
    const char* names[] = {"A <<<>>>", "B hipExtLaunchKernelGGL", "C hipModuleLaunchKernel params", "D hipModuleLaunchKernel extra"};
    for (int form = 0; form < 4; ++form) {
        for (int w = 0; w < 200; ++w) launch(form);
        (void)hipStreamSynchronize(st);
        std::vector<double> per;
        for (int b = 0; b < 10; ++b) {
            for (int i = 0; i < 100; ++i) {
                const auto t0 = clk::now();
                launch(form);
                per.push_back(us(t0, clk::now()));
            }
            (void)hipStreamSynchronize(st);
        }
        // round trip from an idle queue
        std::vector<double> rt;
        a.flag = d;
        for (int i = 0; i < 500; ++i) {
            a.seq = (unsigned long long)(form * 1000000 + i + 1);
            const auto t0 = clk::now();
            launch(form);
            while (*hv != a.seq) {
            }
            if (i > 50) rt.push_back(us(t0, clk::now()));
            (void)hipStreamSynchronize(st);
        }
        a.flag = nullptr;
        std::printf("%-34s launch call median %6.2f us   launch -> kernel flag median %6.2f us\n", names[form], median(per),
                    median(rt));
    }
    return 0;
}
