// Memory-skeleton calibration, round 2 (tool, not product): the classify kernel's per-packet traffic (52 B of the
// 64-B window + the 4-B length read, 4 x 4-B results written) with a tunable amount of dependent VALU work per tile,
// as ONE persistent launch over n packets, for n from 1M to 32M.  Answers: what algorithmic rate does a long launch
// reach, does the non-temporal load / store policy help a once-read stream, and how much per-tile compute does the
// stream hide.
//   hipcc --offload-arch=gfx950 -O3 -o stream_calib2 stream_calib2.hip && ./stream_calib2
#include <hip/hip_runtime.h>
#include <hip/hip_ext.h>
#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e)); exit(1); } } while (0)

struct Args { const uint8_t *hdr; const uint32_t *len; uint32_t n; uint32_t *o0, *o1, *o2, *o3; };

typedef uint32_t v4u __attribute__((ext_vector_type(4)));
template <bool NT> __device__ __forceinline__ uint4 ld4(const uint4 *p) {
    const v4u *q = (const v4u *)p;
    const v4u v = NT ? __builtin_nontemporal_load(q) : *q;
    return make_uint4(v.x, v.y, v.z, v.w);
}
template <bool NT> __device__ __forceinline__ uint32_t ld1(const uint32_t *p) {
    if (NT) return __builtin_nontemporal_load(p);
    return *p;
}
template <bool NT> __device__ __forceinline__ void st1(uint32_t *p, uint32_t v) {
    if (NT) __builtin_nontemporal_store(v, p);
    else *p = v;
}

// row per lane, persistent: wave w takes tiles w, w + W, ...; K rounds of 8 dependent-chain VALU ops per packet
template <bool NTL, bool NTS, int K>
__global__ __launch_bounds__(512) void k_row(Args a) {
    const uint32_t lane = threadIdx.x & 63;
    const uint32_t ntiles = (a.n + 63) >> 6;
    const uint32_t step = gridDim.x * 8;
    for (uint32_t tile = blockIdx.x * 8 + (threadIdx.x >> 6); tile < ntiles; tile += step) {
        const uint32_t p = min(tile * 64 + lane, a.n - 1);
        const uint4 *r = (const uint4 *)(a.hdr + (size_t)p * 64);
        const uint4 q0 = ld4<NTL>(r), q1 = ld4<NTL>(r + 1), q2 = ld4<NTL>(r + 2);
        const uint32_t q3 = ld1<NTL>((const uint32_t *)(r + 3));
        const uint32_t l = ld1<NTL>(a.len + p);
        uint32_t c[8] = {q0.x, q0.y, q0.z, q0.w, q1.x, q1.y, q1.z, q1.w};
#pragma unroll
        for (int k = 0; k < K; ++k)
#pragma unroll
            for (int j = 0; j < 8; ++j) c[j] = (c[j] ^ (c[(j + 1) & 7] >> 3)) + 0x9e3779b9u;
        const uint32_t x = c[0] ^ c[1] ^ c[2] ^ c[3] ^ c[4] ^ c[5] ^ c[6] ^ c[7] ^ q2.x ^ q2.y ^ q2.z ^ q2.w ^ q3;
        st1<NTS>(a.o0 + p, x);
        st1<NTS>(a.o1 + p, x ^ l);
        st1<NTS>(a.o2 + p, x + l);
        st1<NTS>(a.o3 + p, p);
    }
}

typedef void (*KFn)(Args);

int main(int argc, char **argv) {
    hipDeviceProp_t pr;
    CK(hipGetDeviceProperties(&pr, 0));
    const int ncu = pr.multiProcessorCount;
    const uint32_t nmax = 32u << 20;
    // two buffer sets of nmax packets each (2 x 2.8 GB): consecutive launches never re-read what the MALL holds
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
    const V vs[] = {{"plain", k_row<false, false, 0>}, {"ntload", k_row<true, false, 0>},
                    {"ntstore", k_row<false, true, 0>}, {"nt both", k_row<true, true, 0>},
                    {"plain +VALU16", k_row<false, false, 16>}, {"ntload +VALU16", k_row<true, false, 16>},
                    {"plain +VALU32", k_row<false, false, 32>}, {"ntload +VALU32", k_row<true, false, 32>}};
    const uint32_t ns[] = {1u << 20, 2u << 20, 4u << 20, 8u << 20, 16u << 20, 32u << 20};
    const uint32_t grid = (uint32_t)ncu * 4;  // 4 x 512 threads = 32 waves per CU
    for (const V &v : vs) {
        for (uint32_t n : ns) {
            std::vector<float> t;
            const int iters = n >= (8u << 20) ? 10 : 30;
            for (int it = 0; it < iters + 4; ++it) {
                // consecutive launches read distinct chunks (a chunk comes back after >= 2 x 2.8 GB of other traffic)
                Args a = A[it & 1];
                const size_t off = (size_t)((it >> 1) % (nmax / n)) * n;
                a.hdr += off * 64;
                a.len += off;
                a.o0 += off;
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
            printf("%-16s n %5u Mi  med %9.2f us  alg80 %6.1f GB/s  real %6.1f GB/s  us/1M %6.2f\n", v.name, n >> 20,
                   med, 80.0 * n / (med * 1e-6) / 1e9, (68.0 + 16.0) * n / (med * 1e-6) / 1e9, med / (n >> 20));
        }
    }
    return 0;
}
