// Memory-skeleton calibration 4 (tool, not product): C1's per-packet traffic (52 B of the 64-B window + the 4-B
// length read; 16 B written) with the results written as three SoA streams + the list (4 dword stores per lane, the
// engine's layout) or as one 12-B ppe_verdict_t AoS record + the list (a dwordx3 and a dword store per lane).
// Non-temporal stores in both.  One persistent launch over 16M / 32M packets, two buffer sets.
//   hipcc --offload-arch=gfx950 -O3 -o stream_calib4 stream_calib4.hip && ./stream_calib4
#include <hip/hip_runtime.h>
#include <hip/hip_ext.h>
#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e)); exit(1); } } while (0)

struct Args { const uint8_t *hdr; const uint32_t *len; uint32_t n; uint32_t *o0, *o1, *o2, *o3; };
typedef uint32_t v4u __attribute__((ext_vector_type(4)));
typedef uint32_t v3u __attribute__((ext_vector_type(3)));

template <int AOS>
__global__ __launch_bounds__(512) void k_row(Args a) {
    const uint32_t lane = threadIdx.x & 63;
    const uint32_t ntiles = (a.n + 63) >> 6;
    const uint32_t step = gridDim.x * 8;
    for (uint32_t tile = blockIdx.x * 8 + (threadIdx.x >> 6); tile < ntiles; tile += step) {
        const uint32_t p = min(tile * 64 + lane, a.n - 1);
        const v4u *r = (const v4u *)(a.hdr + (size_t)p * 64);
        const v4u q0 = r[0], q1 = r[1], q2 = r[2];
        const uint32_t q3 = *(const uint32_t *)(r + 3);
        const uint32_t l = a.len[p];
        const uint32_t x = q0.x ^ q0.y ^ q0.z ^ q0.w ^ q1.x ^ q1.y ^ q1.z ^ q1.w ^ q2.x ^ q2.y ^ q2.z ^ q2.w ^ q3;
        if (AOS) {
            v3u v = {x, x ^ l, x + l};
            __builtin_nontemporal_store(v, (v3u *)((uint8_t *)a.o0 + 12ull * p));
        } else {
            __builtin_nontemporal_store(x, a.o0 + p);
            __builtin_nontemporal_store(x ^ l, a.o1 + p);
            __builtin_nontemporal_store(x + l, a.o2 + p);
        }
        __builtin_nontemporal_store(p, a.o3 + p);
    }
}

typedef void (*KFn)(Args);

int main() {
    hipDeviceProp_t pr;
    CK(hipGetDeviceProperties(&pr, 0));
    const int ncu = pr.multiProcessorCount;
    const uint32_t nmax = 32u << 20;
    Args A[2];
    for (int b = 0; b < 2; ++b) {
        uint8_t *h;
        uint32_t *l, *o;
        CK(hipMalloc(&h, (size_t)nmax * 64));
        CK(hipMalloc(&l, (size_t)nmax * 4));
        CK(hipMalloc(&o, (size_t)nmax * 16));
        CK(hipMemset(h, b + 1, (size_t)nmax * 64));
        CK(hipMemset(l, 0, (size_t)nmax * 4));
        A[b] = {h, l, nmax, o, o + nmax, o + 2 * (size_t)nmax, o + 3 * (size_t)nmax};
    }
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    struct V { const char *name; KFn fn; };
    const V vs[] = {{"soa x3 + list", k_row<0>}, {"aos12 + list", k_row<1>}};
    const uint32_t grid = (uint32_t)ncu * 4;
    for (int rep = 0; rep < 3; ++rep)
        for (const V &v : vs) {
            for (uint32_t n : {16u << 20, 32u << 20}) {
                std::vector<float> t;
                for (int it = 0; it < 14; ++it) {
                    Args a = A[it & 1];
                    const size_t off = (size_t)((it >> 1) % (nmax / n)) * n;
                    a.hdr += off * 64;
                    a.len += off;
                    a.o0 += off * (v.fn == k_row<1> ? 3 : 1);
                    a.o1 += off;
                    a.o2 += off;
                    a.o3 += off;
                    a.n = n;
                    hipEvent_t s = it >= 4 ? e0 : nullptr, f = it >= 4 ? e1 : nullptr;
                    hipExtLaunchKernelGGL(v.fn, dim3(grid), dim3(512), 0, 0, s, f, 0, a);
                    if (it >= 4) {
                        CK(hipEventSynchronize(e1));
                        float ms;
                        CK(hipEventElapsedTime(&ms, e0, e1));
                        t.push_back(ms);
                    }
                }
                std::sort(t.begin(), t.end());
                const double med = t[t.size() / 2] * 1e3;
                printf("%-16s n %5u Mi  med %9.2f us  alg80 %6.1f GB/s  us/1M %6.2f\n", v.name, n >> 20, med,
                       80.0 * n / (med * 1e-6) / 1e9, med / (n >> 20));
            }
        }
    return 0;
}
