// Host-decision -> kernel-start latency, three ways (diagnostics for DESIGN §8):
//  A. the host launches the next kernel after its decision (what lio_match does);
//  B. the kernel was enqueued beforehand behind hipStreamWaitValue64 on a host-mapped word,
//     the host's decision is one store to that word;
//  C. the kernel was enqueued beforehand and its single block spins on the host-mapped word
//     (bounded spin: gives up after ~20 ms so a lost store cannot hang the queue).
// Each round trip: host t0 -> (launch | store) -> kernel writes seq to a host-mapped flag ->
// host sees it.  Reports the median / p90 in microseconds.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <thread>
#include <vector>

typedef __attribute__((address_space(1))) unsigned long long gull;

__global__ void k_flag(unsigned long long* out, unsigned long long seq) {
    if (threadIdx.x == 0) __hip_atomic_store((gull*)out, seq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}
__global__ void k_spin_flag(const unsigned long long* in, unsigned long long* out, unsigned long long seq) {
    if (threadIdx.x == 0) {
        const unsigned long long t0 = wall_clock64();
        while (__hip_atomic_load((gull*)in, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) < seq) {
            if (wall_clock64() - t0 > 2000000ull) break;  // 100 MHz wall clock: 20 ms
            __builtin_amdgcn_s_sleep(1);
        }
        __hip_atomic_store((gull*)out, seq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    }
}

__global__ void k_busy(unsigned long long ticks) {  // one wave busy for `ticks` of the 100 MHz clock
    const unsigned long long t0 = wall_clock64();
    while (wall_clock64() - t0 < ticks) __builtin_amdgcn_s_sleep(1);
}

static void report(const char* name, std::vector<double>& v) {
    std::sort(v.begin(), v.end());
    std::printf("%-44s median %7.2f us  p10 %7.2f  p90 %7.2f  (n=%zu)\n", name, v[v.size() / 2], v[v.size() / 10],
                v[v.size() * 9 / 10], v.size());
}

int main() {
    using clk = std::chrono::steady_clock;
    hipStream_t st;
    (void)hipStreamCreateWithFlags(&st, hipStreamNonBlocking);
    unsigned long long *h, *d;
    (void)hipHostMalloc(&h, 256, hipHostMallocMapped | hipHostMallocCoherent);
    (void)hipHostGetDevicePointer((void**)&d, h, 0);
    volatile unsigned long long* hin = h;       // host -> device word
    volatile unsigned long long* hout = h + 8;  // device -> host word
    unsigned long long* din = d;
    unsigned long long* dout = d + 8;
    *hin = 0;
    *hout = 0;
    const int N = 3000;
    unsigned long long seq = 0;
    auto us = [](clk::time_point a, clk::time_point b) { return std::chrono::duration<double, std::micro>(b - a).count(); };
    std::vector<double> va, vb, vc;
    for (int it = 0; it < N; ++it) {  // A
        ++seq;
        const auto t0 = clk::now();
        k_flag<<<1, 64, 0, st>>>(dout, seq);
        while (*hout != seq) {
        }
        if (it > 100) va.push_back(us(t0, clk::now()));
    }
    (void)hipStreamSynchronize(st);
    bool have_wait = true;
    for (int it = 0; it < N && have_wait; ++it) {  // B
        ++seq;
        if (hipStreamWaitValue64(st, din, seq, hipStreamWaitValueGte, ~0ull) != hipSuccess) {
            std::printf("hipStreamWaitValue64 unsupported: %s\n", hipGetErrorString(hipGetLastError()));
            have_wait = false;
            break;
        }
        k_flag<<<1, 64, 0, st>>>(dout, seq);
        std::this_thread::sleep_for(std::chrono::microseconds(30));  // the queue is parked on the wait
        const auto t0 = clk::now();
        *hin = seq;
        while (*hout != seq) {
        }
        if (it > 100) vb.push_back(us(t0, clk::now()));
    }
    (void)hipStreamSynchronize(st);
    for (int it = 0; it < N; ++it) {  // C
        ++seq;
        k_spin_flag<<<1, 64, 0, st>>>(din, dout, seq);
        std::this_thread::sleep_for(std::chrono::microseconds(30));
        const auto t0 = clk::now();
        *hin = seq;
        while (*hout != seq) {
        }
        if (it > 100) vc.push_back(us(t0, clk::now()));
    }
    (void)hipStreamSynchronize(st);
    // D: the host's store lands BEFORE the spinning gate starts (it is queued behind a 20 us kernel),
    // as in lio_ieskf_update; time from the store to the gate's completion minus the busy kernel
    std::vector<double> vd;
    for (int it = 0; it < N; ++it) {
        ++seq;
        k_busy<<<1, 64, 0, st>>>(2000);  // 20 us
        k_spin_flag<<<1, 64, 0, st>>>(din, dout, seq);
        const auto t0 = clk::now();
        *hin = seq;
        while (*hout != seq) {
        }
        if (it > 100) vd.push_back(us(t0, clk::now()));
    }
    (void)hipStreamSynchronize(st);
    // E / F: as D, but the host first writes a 576-byte payload next to the word (the gate block of
    // lio_capi.cpp: seq, cmd, two poses), without (E) and with (F) an mfence after the word
    unsigned long long *g, *gd;
    (void)hipHostMalloc(&g, 1024, hipHostMallocMapped | hipHostMallocCoherent);
    (void)hipHostGetDevicePointer((void**)&gd, g, 0);
    std::vector<double> ve, vf;
    for (int pass = 0; pass < 2; ++pass) {
        for (int it = 0; it < N; ++it) {
            ++seq;
            k_busy<<<1, 64, 0, st>>>(2000);
            k_spin_flag<<<1, 64, 0, st>>>(gd, dout, seq);
            const auto t0 = clk::now();
            volatile double* pl = reinterpret_cast<volatile double*>(g + 2);
            for (int k = 0; k < 72; ++k) pl[k] = (double)(seq + k);
            reinterpret_cast<volatile unsigned long long*>(g)[1] = 1;
            reinterpret_cast<volatile unsigned long long*>(g)[0] = seq;
            if (pass == 1) __builtin_ia32_mfence();
            while (*hout != seq) {
            }
            if (it > 100) (pass ? vf : ve).push_back(us(t0, clk::now()));
        }
        (void)hipStreamSynchronize(st);
    }
    report("A launch after the decision", va);
    if (have_wait) report("B pre-enqueued behind hipStreamWaitValue64", vb);
    report("C pre-enqueued, one block spinning", vc);
    report("D store before the gate starts (incl. 20 us busy)", vd);
    report("E as D after a 576-B payload (incl. 20 us busy)", ve);
    report("F as E + mfence (incl. 20 us busy)", vf);
    return 0;
}
