// Memory-skeleton calibration for the classify kernel (tool, not product): the same per-packet traffic as
// ppe_classify_kernel (64-B header window + 4-B length read, 4 × 4-B SoA results written) with trivial compute,
// under different load shapes / grid shapes.  Gives the practical HBM ceiling for the C1 workload on this box.
//   hipcc --offload-arch=gfx950 -O3 -o stream_calib stream_calib.hip && ./stream_calib [n_pkts] [nbufs]
#include <hip/hip_runtime.h>
#include <hip/hip_ext.h>
#include <cstdio>
#include <cstdlib>
#include <vector>
#include <algorithm>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e)); exit(1); } } while (0)

struct Args { const uint8_t *hdr; const uint32_t *len; uint32_t n; uint32_t *o0, *o1, *o2, *o3; };

__device__ __forceinline__ void emit(const Args &a, uint32_t p, uint32_t x, uint32_t l) {
    a.o0[p] = x; a.o1[p] = x ^ l; a.o2[p] = x + l; a.o3[p] = p;
}

// 1. row per lane (what the classify kernel does): lane = packet, 4 × 16-B loads at stride 64
template <bool PERSIST>
__global__ __launch_bounds__(256) void k_row(Args a) {
    const uint32_t lane = threadIdx.x & 63;
    const uint32_t ntiles = (a.n + 63) >> 6;
    uint32_t tile = blockIdx.x * 4 + (threadIdx.x >> 6);
    const uint32_t step = PERSIST ? gridDim.x * 4 : ntiles;
    for (; tile < ntiles; tile += step) {
        const uint32_t p = tile * 64 + lane;
        if (p >= a.n) continue;
        const uint4 *r = (const uint4 *)(a.hdr + (size_t)p * 64);
        const uint4 q0 = r[0], q1 = r[1], q2 = r[2], q3 = r[3];
        const uint32_t l = a.len[p];
        const uint32_t x = q0.x ^ q0.y ^ q0.z ^ q0.w ^ q1.x ^ q1.y ^ q1.z ^ q1.w ^ q2.x ^ q2.y ^ q2.z ^ q2.w ^
                           q3.x ^ q3.y ^ q3.z ^ q3.w;
        emit(a, p, x, l);
    }
}

// 1b. row per lane + K rounds of dummy VALU work per packet (8 independent chains, ~2 instr per chain per round):
// how much per-tile compute the HBM stream hides
template <int K>
__global__ __launch_bounds__(256) void k_rowc(Args a) {
    const uint32_t lane = threadIdx.x & 63;
    const uint32_t ntiles = (a.n + 63) >> 6;
    uint32_t tile = blockIdx.x * 4 + (threadIdx.x >> 6);
    const uint32_t step = gridDim.x * 4;
    for (; tile < ntiles; tile += step) {
        const uint32_t p = tile * 64 + lane;
        if (p >= a.n) continue;
        const uint4 *r = (const uint4 *)(a.hdr + (size_t)p * 64);
        const uint4 q0 = r[0], q1 = r[1], q2 = r[2], q3 = r[3];
        const uint32_t l = a.len[p];
        uint32_t c[8] = {q0.x, q0.y, q0.z, q0.w, q1.x, q1.y, q1.z, q1.w};
#pragma unroll
        for (int k = 0; k < K; ++k)
#pragma unroll
            for (int j = 0; j < 8; ++j) c[j] = (c[j] ^ (c[(j + 1) & 7] >> 3)) + 0x9e3779b9u;
        const uint32_t x = c[0] ^ c[1] ^ c[2] ^ c[3] ^ c[4] ^ c[5] ^ c[6] ^ c[7] ^ q2.x ^ q3.y;
        emit(a, p, x, l);
    }
}

// 2. coalesced: each 16-B load instruction covers 1 KB contiguous; the packet's 64 B end up in 4 lanes, gathered
// back with an LDS transpose (row-per-lane afterwards, like the classify kernel needs)
template <bool PERSIST>
__global__ __launch_bounds__(256) void k_coal(Args a) {
    __shared__ uint4 buf[4][64 * 4 + 4];
    const uint32_t lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const uint32_t ntiles = (a.n + 63) >> 6;
    uint32_t tile = blockIdx.x * 4 + wv;
    const uint32_t step = PERSIST ? gridDim.x * 4 : ntiles;
    for (; tile < ntiles; tile += step) {
        const uint4 *t = (const uint4 *)(a.hdr + (size_t)tile * 4096);
        uint4 c[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) c[k] = t[k * 64 + lane];  // tile is full for these sizes
        const uint32_t p = tile * 64 + lane;
        const uint32_t l = a.len[p];
#pragma unroll
        for (int k = 0; k < 4; ++k) { uint32_t i = k * 64 + lane; buf[wv][i + (i >> 6)] = c[k]; }
        __builtin_amdgcn_wave_barrier();
        uint4 q[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) { uint32_t i = lane * 4 + k; q[k] = buf[wv][i + (i >> 6)]; }
        __builtin_amdgcn_wave_barrier();
        uint32_t x = 0;
#pragma unroll
        for (int k = 0; k < 4; ++k) x ^= q[k].x ^ q[k].y ^ q[k].z ^ q[k].w;
        emit(a, p, x, l);
    }
}

// 4. tile-transposed (AoSoA) layout: per 64-packet tile, 16 planes of 64 dwords; lane reads dword k of its own
// packet with perfectly coalesced 256-B dword loads (no transpose needed)
template <bool PERSIST>
__global__ __launch_bounds__(256) void k_soa(Args a) {
    const uint32_t lane = threadIdx.x & 63;
    const uint32_t ntiles = (a.n + 63) >> 6;
    uint32_t tile = blockIdx.x * 4 + (threadIdx.x >> 6);
    const uint32_t step = PERSIST ? gridDim.x * 4 : ntiles;
    for (; tile < ntiles; tile += step) {
        const uint32_t *t = (const uint32_t *)(a.hdr + (size_t)tile * 4096);
        uint32_t x = 0;
#pragma unroll
        for (int k = 0; k < 16; ++k) x ^= t[k * 64 + lane];
        const uint32_t p = tile * 64 + lane;
        emit(a, p, x, a.len[p]);
    }
}

// 5. LDS-DMA: four global_load_lds_dwordx4 per tile (1 KB each, contiguous) into a per-wave 4-KB LDS slot, then
// row-per-lane ds_read_b128 with a per-lane chunk rotation (conflict-free), double-buffered: tile t+1's DMA is in
// flight while tile t is read
template <int NBUF>
__global__ __launch_bounds__(256) void k_dma(Args a) {
    typedef __attribute__((address_space(1))) const void *gptr_t;
    typedef __attribute__((address_space(3))) void *lptr_t;
    __shared__ __attribute__((aligned(16))) uint32_t buf[4][NBUF][1024 + 64];  // 4 KB window tile + 256 B lens
    const uint32_t lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const uint32_t ntiles = (a.n + 63) >> 6;
    uint32_t tile = blockIdx.x * 4 + wv;
    const uint32_t step = gridDim.x * 4;
    auto issue = [&](uint32_t t, int b) {
        const uint32_t tt = min(t, ntiles - 1);
        const uint4 *g = (const uint4 *)(a.hdr + (size_t)tt * 4096);
#pragma unroll
        for (int k = 0; k < 4; ++k)
            __builtin_amdgcn_global_load_lds((gptr_t)(g + k * 64 + lane), (lptr_t)(&buf[wv][b][k * 256]), 16, 0, 0);
        __builtin_amdgcn_global_load_lds((gptr_t)(a.len + tt * 64 + lane), (lptr_t)(&buf[wv][b][1024]), 4, 0, 0);
    };
#pragma unroll
    for (int b = 0; b < NBUF - 1; ++b) issue(tile + b * step, b);
    int b = 0;
    for (; tile < ntiles; tile += step) {
        issue(tile + (NBUF - 1) * step, (b + NBUF - 1) % NBUF);
        const uint32_t p = tile * 64 + lane;
        // wait until this tile's 5 DMA ops have landed; newer ones: (NBUF-1) x (5 DMA + 4 stores)
        if (NBUF == 2) asm volatile("s_waitcnt vmcnt(9)" ::: "memory");
        else asm volatile("s_waitcnt vmcnt(18)" ::: "memory");
        // ds_read in asm: the compiler would otherwise put vmcnt(0) before any LDS read (it cannot tell which LDS
        // bytes the in-flight DMA writes)
        const uint32_t base = (uint32_t)(uintptr_t)(lptr_t)&buf[wv][b][lane * 16];
        const uint32_t r0 = base + (((0 + (lane >> 2)) & 3) << 4), r1 = base + (((1 + (lane >> 2)) & 3) << 4);
        const uint32_t r2 = base + (((2 + (lane >> 2)) & 3) << 4), r3 = base + (((3 + (lane >> 2)) & 3) << 4);
        const uint32_t rl = (uint32_t)(uintptr_t)(lptr_t)&buf[wv][b][1024 + lane];
        typedef uint32_t v4u __attribute__((ext_vector_type(4)));
        v4u q0, q1, q2, q3;
        uint32_t l;
        asm volatile("ds_read_b128 %0, %5\n\tds_read_b128 %1, %6\n\tds_read_b128 %2, %7\n\tds_read_b128 %3, %8\n\t"
                     "ds_read_b32 %4, %9\n\ts_waitcnt lgkmcnt(0)"
                     : "=&v"(q0), "=&v"(q1), "=&v"(q2), "=&v"(q3), "=&v"(l)
                     : "v"(r0), "v"(r1), "v"(r2), "v"(r3), "v"(rl) : "memory");
        uint32_t x = q0.x ^ q0.y ^ q0.z ^ q0.w ^ q1.x ^ q1.y ^ q1.z ^ q1.w ^ q2.x ^ q2.y ^ q2.z ^ q2.w ^ q3.x ^ q3.y ^
                     q3.z ^ q3.w;
        emit(a, p, x, l);
        b = (b + 1) % NBUF;
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

// 3. plain copy-like: one dwordx4 per lane, contiguous (upper bound for this byte count)
__global__ __launch_bounds__(256) void k_flat(Args a) {
    const size_t nv = (size_t)a.n * 4;  // 16-B vectors of header data
    const uint4 *h = (const uint4 *)a.hdr;
    for (size_t i = blockIdx.x * 256 + threadIdx.x; i < nv; i += (size_t)gridDim.x * 256) {
        const uint4 q = h[i];
        const uint32_t x = q.x ^ q.y ^ q.z ^ q.w;
        if ((i & 3) == 0) { const uint32_t p = i >> 2; emit(a, p, x, a.len[p]); }
    }
}

int main(int argc, char **argv) {
    const uint32_t n = argc > 1 ? atoi(argv[1]) : (1u << 20);
    const int nb = argc > 2 ? atoi(argv[2]) : 4;
    hipDeviceProp_t pr; CK(hipGetDeviceProperties(&pr, 0));
    const int ncu = pr.multiProcessorCount;
    std::vector<Args> A(nb);
    for (int b = 0; b < nb; ++b) {
        uint8_t *h; uint32_t *l, *o;
        CK(hipMalloc(&h, (size_t)n * 64)); CK(hipMalloc(&l, (size_t)n * 4)); CK(hipMalloc(&o, (size_t)n * 16));
        CK(hipMemset(h, b + 1, (size_t)n * 64)); CK(hipMemset(l, 0, (size_t)n * 4));
        A[b] = {h, l, n, o, o + n, o + 2 * (size_t)n, o + 3 * (size_t)n};
    }
    const double bytes = (double)n * (64 + 4 + 16);
    hipEvent_t e0, e1; CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
    struct V { const char *name; int which; uint32_t grid; };
    const uint32_t tiles = (n + 63) / 64;
    V vs[] = {{"row  1tile/wave", 0, (tiles + 3) / 4}, {"row  persist 8/CU", 1, (uint32_t)ncu * 8},
              {"row  persist 4/CU", 1, (uint32_t)ncu * 4}, {"row  persist 16/CU", 1, (uint32_t)ncu * 16},
              {"coal 1tile/wave", 2, (tiles + 3) / 4}, {"coal persist 8/CU", 3, (uint32_t)ncu * 8},
              {"flat persist 8/CU", 4, (uint32_t)ncu * 8}, {"flat 1 vec/thread", 4, (n * 4 + 255) / 256},
              {"soa  1tile/wave", 5, (tiles + 3) / 4}, {"soa  persist 8/CU", 6, (uint32_t)ncu * 8},
              {"dma2 persist 4/CU", 7, (uint32_t)ncu * 4}, {"dma2 persist 8/CU", 7, (uint32_t)ncu * 8},
              {"dma3 persist 4/CU", 8, (uint32_t)ncu * 4},
              {"row+VALU x8 (~200/tile)", 9, (uint32_t)ncu * 8}, {"row+VALU x16 (~400/tile)", 10, (uint32_t)ncu * 8},
              {"row+VALU x32 (~800/tile)", 11, (uint32_t)ncu * 8}, {"row+VALU x64 (~1600/tile)", 12, (uint32_t)ncu * 8}};
    const int iters = 200;
    for (const V &v : vs) {
        std::vector<float> t;
        for (int it = 0; it < iters + 20; ++it) {
            const Args &a = A[it % nb];
            hipEvent_t s = it >= 20 ? e0 : nullptr, f = it >= 20 ? e1 : nullptr;
            switch (v.which) {
            case 0: hipExtLaunchKernelGGL(k_row<false>, dim3(v.grid), dim3(256), 0, 0, s, f, 0, a); break;
            case 1: hipExtLaunchKernelGGL(k_row<true>, dim3(v.grid), dim3(256), 0, 0, s, f, 0, a); break;
            case 2: hipExtLaunchKernelGGL(k_coal<false>, dim3(v.grid), dim3(256), 0, 0, s, f, 0, a); break;
            case 3: hipExtLaunchKernelGGL(k_coal<true>, dim3(v.grid), dim3(256), 0, 0, s, f, 0, a); break;
            case 4: hipExtLaunchKernelGGL(k_flat, dim3(v.grid), dim3(256), 0, 0, s, f, 0, a); break;
            case 5: hipExtLaunchKernelGGL(k_soa<false>, dim3(v.grid), dim3(256), 0, 0, s, f, 0, a); break;
            case 6: hipExtLaunchKernelGGL(k_soa<true>, dim3(v.grid), dim3(256), 0, 0, s, f, 0, a); break;
            case 7: hipExtLaunchKernelGGL(k_dma<2>, dim3(v.grid), dim3(256), 0, 0, s, f, 0, a); break;
            case 8: hipExtLaunchKernelGGL(k_dma<3>, dim3(v.grid), dim3(256), 0, 0, s, f, 0, a); break;
            case 9: hipExtLaunchKernelGGL(k_rowc<8>, dim3(v.grid), dim3(256), 0, 0, s, f, 0, a); break;
            case 10: hipExtLaunchKernelGGL(k_rowc<16>, dim3(v.grid), dim3(256), 0, 0, s, f, 0, a); break;
            case 11: hipExtLaunchKernelGGL(k_rowc<32>, dim3(v.grid), dim3(256), 0, 0, s, f, 0, a); break;
            case 12: hipExtLaunchKernelGGL(k_rowc<64>, dim3(v.grid), dim3(256), 0, 0, s, f, 0, a); break;
            }
            if (it >= 20) { CK(hipEventSynchronize(e1)); float ms; CK(hipEventElapsedTime(&ms, e0, e1)); t.push_back(ms); }
        }
        std::sort(t.begin(), t.end());
        const double med = t[t.size() / 2] * 1e3, mn = t[0] * 1e3;
        printf("%-22s grid %6u  med %7.2f us  min %7.2f us  %7.1f GB/s (med)\n", v.name, v.grid, med, mn, bytes / (med * 1e-6) / 1e9);
    }
    // back-to-back throughput (no per-launch events) for the row/persist shape
    for (int w = 0; w < 2; ++w) {
        const uint32_t grid = (uint32_t)ncu * 8;
        CK(hipDeviceSynchronize());
        CK(hipEventRecord(e0, 0));
        for (int it = 0; it < iters; ++it) hipLaunchKernelGGL(w ? k_flat : k_row<true>, dim3(grid), dim3(256), 0, 0, A[it % nb]);
        CK(hipEventRecord(e1, 0)); CK(hipEventSynchronize(e1));
        float ms; CK(hipEventElapsedTime(&ms, e0, e1));
        printf("back-to-back %s: %.2f us/launch  %.1f GB/s\n", w ? "flat" : "row persist", ms * 1e3 / iters, bytes * iters / (ms * 1e-3) / 1e9);
    }
    // the same launches alternating over two streams (consecutive launches overlap, like ppe_classify_batches)
    {
        hipStream_t s2[2];
        hipEvent_t ej[2];
        for (int k = 0; k < 2; ++k) {
            CK(hipStreamCreateWithFlags(&s2[k], hipStreamNonBlocking));
            CK(hipEventCreate(&ej[k]));
        }
        for (int w = 0; w < 2; ++w) {
            const uint32_t grid = (uint32_t)ncu * 8;
            CK(hipDeviceSynchronize());
            CK(hipEventRecord(e0, 0));
            for (int k = 0; k < 2; ++k) CK(hipStreamWaitEvent(s2[k], e0, 0));
            for (int it = 0; it < iters; ++it)
                hipLaunchKernelGGL(w ? k_flat : k_row<true>, dim3(grid), dim3(256), 0, s2[it & 1], A[it % nb]);
            for (int k = 0; k < 2; ++k) {
                CK(hipEventRecord(ej[k], s2[k]));
                CK(hipStreamWaitEvent(0, ej[k], 0));
            }
            CK(hipEventRecord(e1, 0)); CK(hipEventSynchronize(e1));
            float ms; CK(hipEventElapsedTime(&ms, e0, e1));
            printf("two-stream %s: %.2f us/launch  %.1f GB/s\n", w ? "flat" : "row persist", ms * 1e3 / iters, bytes * iters / (ms * 1e-3) / 1e9);
        }
    }
    return 0;
}
