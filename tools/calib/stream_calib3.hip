// Memory-skeleton calibration, round 2b (tool, not product): how a wave should fetch its 64-packet tile.
// The per-lane row loads of the classify kernel (4 loads per lane at a 64-B row stride: every wave-instruction touches
// 32 cache lines) keep the TA/TD path ~90 % busy (r2zf: TD_BUSY 564 cycles per tile).  Here the same traffic (64-B
// windows, 4-B lengths, 4 x 4-B results per packet) is fetched
//   row     as the classify kernel does today (row per lane, 8 waves/SIMD)
//   dma*    as 4 coalesced 1-KiB LDS-DMA pieces per tile (global_load_lds_dwordx4), each row's 16-B chunks permuted
//           by XOR ((row >> 2) & 3) through the per-lane source address, then read back row-per-lane with 4
//           conflict-free ds_read_b128 (lane r: 64 r + 16 (c ^ ((r >> 2) & 3)))
//   single buffer (DMA, wait, read), or double buffer (next tile's DMA in flight while the current one is used),
//   at 16 or 32 waves per CU.
//   hipcc --offload-arch=gfx950 -O3 -o stream_calib3 stream_calib3.hip && ./stream_calib3
#include <hip/hip_runtime.h>
#include <hip/hip_ext.h>
#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e)); exit(1); } } while (0)

struct Args { const uint8_t *hdr; const uint32_t *len; uint32_t n; uint32_t *o0, *o1, *o2, *o3; uint32_t *chk; };
typedef __attribute__((address_space(1))) const void *gptr_t;
typedef __attribute__((address_space(3))) void *lptr_t;

__device__ __forceinline__ void st_nt(uint32_t *p, uint32_t v) { __builtin_nontemporal_store(v, p); }

__device__ __forceinline__ uint32_t work(uint4 q0, uint4 q1, uint4 q2, uint32_t q3) {
    return q0.x ^ q0.y ^ q0.z ^ q0.w ^ q1.x ^ q1.y ^ q1.z ^ q1.w ^ q2.x ^ q2.y ^ q2.z ^ q2.w ^ q3;
}

__device__ __forceinline__ void put(const Args &a, uint32_t p, uint32_t x, uint32_t l, bool valid) {
    if (!valid) return;
    st_nt(a.o0 + p, x);
    st_nt(a.o1 + p, x ^ l);
    st_nt(a.o2 + p, x + l);
    st_nt(a.o3 + p, p);
}

template <int WPB>
__global__ __launch_bounds__(64 * WPB) void k_row(Args a) {
    const uint32_t lane = threadIdx.x & 63;
    const uint32_t ntiles = (a.n + 63) >> 6;
    const uint32_t step = gridDim.x * WPB;
    for (uint32_t tile = blockIdx.x * WPB + (threadIdx.x >> 6); tile < ntiles; tile += step) {
        const uint32_t p = min(tile * 64 + lane, a.n - 1);
        const uint4 *r = (const uint4 *)(a.hdr + (size_t)p * 64);
        const uint4 q0 = r[0], q1 = r[1], q2 = r[2];
        const uint32_t q3 = *(const uint32_t *)(r + 3);
        const uint32_t l = a.len[p];
        put(a, tile * 64 + lane, work(q0, q1, q2, q3), l, tile * 64 + lane < a.n);
    }
}

// one 1-KiB LDS-DMA piece, hidden from the compiler's waitcnt model (it would put vmcnt(0) before every LDS read):
// the kernel waits for the pieces itself with a counted s_waitcnt vmcnt
__device__ __forceinline__ void dma16(const void *src, uint32_t lds_byte) {
    uint32_t keep;
    asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
                 : "=&s"(keep) : "v"(src), "s"(lds_byte) : "memory");
}

// the 4 DMA pieces of one tile into the wave's 4-KiB LDS slot (row-chunk XOR permutation on the source side)
template <bool ASM = false>
__device__ __forceinline__ void dma_tile(const Args &a, uint32_t tile, uint32_t lane, uint32_t *slot) {
    const uint32_t base = __builtin_amdgcn_readfirstlane((uint32_t)(size_t)(lptr_t)slot);
#pragma unroll
    for (uint32_t j = 0; j < 4; ++j) {
        const uint32_t row = 16u * j + (lane >> 2);
        const uint32_t chunk = (lane & 3u) ^ ((lane >> 4) & 3u);
        const uint32_t p = min(tile * 64u + row, a.n - 1u);
        const uint8_t *src = a.hdr + (size_t)p * 64 + 16u * chunk;
        if (ASM)
            dma16(src, base + 1024u * j);
        else
            __builtin_amdgcn_global_load_lds((gptr_t)src, (lptr_t)(slot + 256u * j), 16, 0, 0);
    }
}

__device__ __forceinline__ void read_rows(const uint32_t *slot, uint32_t lane, uint4 &q0, uint4 &q1, uint4 &q2,
                                          uint32_t &q3) {
    const uint32_t f = (lane >> 2) & 3u;
    const uint4 *r = (const uint4 *)(slot + 16u * lane);
    q0 = r[0u ^ f];
    q1 = r[1u ^ f];
    q2 = r[2u ^ f];
    q3 = r[3u ^ f].x;
}

template <int WPB>
__global__ __launch_bounds__(64 * WPB) void k_dma1(Args a) {
    __shared__ uint32_t lds[WPB][1024];
    const uint32_t lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const uint32_t ntiles = (a.n + 63) >> 6;
    const uint32_t step = gridDim.x * WPB;
    for (uint32_t tile = blockIdx.x * WPB + w; tile < ntiles; tile += step) {
        dma_tile(a, tile, lane, lds[w]);
        const uint32_t l = a.len[min(tile * 64 + lane, a.n - 1)];
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        uint4 q0, q1, q2;
        uint32_t q3;
        read_rows(lds[w], lane, q0, q1, q2, q3);
        put(a, tile * 64 + lane, work(q0, q1, q2, q3), l, tile * 64 + lane < a.n);
    }
}

__device__ __forceinline__ void dma4(const void *src, uint32_t lds_byte) {
    uint32_t keep;
    asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dword %1, off\n\ts_mov_b32 m0, %0"
                 : "=&s"(keep) : "v"(src), "s"(lds_byte) : "memory");
}

// tile + its 64 lengths (a 5th DMA piece of 256 B): nothing the loop carries is a pending VGPR load, so the compiler
// puts no vmcnt(0) at the back edge
template <int WPB, int NW = 5>
__global__ __launch_bounds__(64 * WPB) void k_dma2(Args a) {
    __shared__ uint32_t lds[WPB][2][1024 + 64];
    const uint32_t lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const uint32_t ntiles = (a.n + 63) >> 6;
    const uint32_t step = gridDim.x * WPB;
    uint32_t tile = blockIdx.x * WPB + w;
    auto issue = [&](uint32_t t, uint32_t *slot) {
        dma_tile<true>(a, t, lane, slot);
        dma4(a.len + min(t * 64 + lane, a.n - 1), __builtin_amdgcn_readfirstlane((uint32_t)(size_t)(lptr_t)(slot + 1024)));
    };
    if (tile < ntiles) issue(tile, lds[w][0]);
    for (uint32_t k = 0; tile < ntiles; tile += step, ++k) {
        const uint32_t next = tile + step;
        if (next < ntiles) {
            issue(next, lds[w][(k + 1) & 1]);
            // this tile's pieces (and its length) have landed: NW = the next tile's 4 pieces + its lengths (5), + the
            // previous tile's 4 result stores (9)
            if (NW == 9) asm volatile("s_waitcnt vmcnt(9)" ::: "memory");
            else asm volatile("s_waitcnt vmcnt(5)" ::: "memory");
        } else {
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        }
        uint4 q0, q1, q2;
        uint32_t q3;
        read_rows(lds[w][k & 1], lane, q0, q1, q2, q3);
        const uint32_t l = lds[w][k & 1][1024 + lane];
        put(a, tile * 64 + lane, work(q0, q1, q2, q3), l, tile * 64 + lane < a.n);
    }
}

typedef void (*KFn)(Args);

__global__ void k_check(const uint8_t *hdr, uint32_t n, const uint32_t *o0, uint32_t *bad) {
    const uint32_t p = blockIdx.x * blockDim.x + threadIdx.x;
    if (p >= n) return;
    const uint32_t *r = (const uint32_t *)(hdr + (size_t)p * 64);
    uint32_t x = 0;
    for (int i = 0; i < 13; ++i) x ^= r[i];
    if (o0[p] != x) atomicAdd(bad, 1u);
}

int main(int argc, char **argv) {
    hipDeviceProp_t pr;
    CK(hipGetDeviceProperties(&pr, 0));
    const int ncu = pr.multiProcessorCount;
    const uint32_t nmax = 32u << 20;
    Args A[2];
    uint32_t *bad;
    CK(hipMalloc(&bad, 4));
    for (int b = 0; b < 2; ++b) {
        uint8_t *h;
        uint32_t *l, *o;
        CK(hipMalloc(&h, (size_t)nmax * 64));
        CK(hipMalloc(&l, (size_t)nmax * 4));
        CK(hipMalloc(&o, (size_t)nmax * 16));
        std::vector<uint32_t> hv((size_t)nmax * 16);
        uint32_t s = 12345u + b;
        for (auto &v : hv) v = (s = s * 1664525u + 1013904223u);
        CK(hipMemcpy(h, hv.data(), (size_t)nmax * 64, hipMemcpyHostToDevice));
        CK(hipMemset(l, 0, (size_t)nmax * 4));
        A[b] = {h, l, nmax, o, o + nmax, o + 2 * (size_t)nmax, o + 3 * (size_t)nmax, bad};
    }
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    struct V { const char *name; KFn fn; int block, per_cu; };
    const V vs[] = {{"row 32w", k_row<8>, 512, 4},          {"dma1 16w", k_dma1<16>, 1024, 1},
                    {"dma1 32w", k_dma1<8>, 512, 4},        {"dma2 16w", k_dma2<16>, 1024, 1},
                    {"dma2 12w", k_dma2<12>, 768, 1},       {"dma1 24w", k_dma1<12>, 768, 2},
                    {"dma2 8w", k_dma2<8>, 512, 1},         {"dma2s 16w", k_dma2<16, 9>, 1024, 1},
                    {"dma2s 12w", k_dma2<12, 9>, 768, 1}};
    const uint32_t ns[] = {4u << 20, 32u << 20};
    for (const V &v : vs) {
        const uint32_t grid = (uint32_t)ncu * v.per_cu;
        for (uint32_t n : ns) {
            std::vector<float> t;
            const int iters = n >= (8u << 20) ? 10 : 30;
            for (int it = 0; it < iters + 4; ++it) {
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
                hipExtLaunchKernelGGL(v.fn, dim3(grid), dim3(v.block), 0, 0, s, f, 0, a);
                if (it >= 4) {
                    CK(hipEventSynchronize(e1));
                    float ms;
                    CK(hipEventElapsedTime(&ms, e0, e1));
                    t.push_back(ms);
                }
                if (it == 0) {
                    CK(hipMemset(bad, 0, 4));
                    hipLaunchKernelGGL(k_check, dim3((n + 255) / 256), dim3(256), 0, 0, a.hdr, n, a.o0, bad);
                    uint32_t nb = 0;
                    CK(hipMemcpy(&nb, bad, 4, hipMemcpyDeviceToHost));
                    if (nb) printf("%s: %u wrong results\n", v.name, nb);
                }
            }
            std::sort(t.begin(), t.end());
            const double med = t[t.size() / 2] * 1e3;
            printf("%-10s n %3u Mi  med %9.2f us  alg80 %6.1f GB/s  us/1M %6.2f\n", v.name, n >> 20, med,
                   80.0 * n / (med * 1e-6) / 1e9, med / (n >> 20));
        }
    }
    return 0;
}
