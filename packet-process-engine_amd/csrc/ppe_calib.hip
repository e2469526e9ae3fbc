/*
 * ppe_calib.hip — same-run memory ceilings for bench.py's roofline (measurement only, not the product path; built as
 * libppe_calib.so next to libppe_hip.so).
 *
 *   skeleton    the classify kernel's own HBM traffic and launch shape with no decode / ACL work: per packet the first
 *               52 B of the 64-B window and the 4-B length read, four 4-B results written (verdict, flow hash, ACL
 *               hit, partition entry), one packet per lane, 64-packet tiles, a persistent grid over up to 32 batches
 *               in one launch (the ring launch of ppe_classify_batches)
 *   read-only   the same reads, one 4-B word written per 64-packet tile: separates the write mix from the row fetch
 *   skel-12+1   (mode 2) the skeleton with a 1-B partition entry (tile offset | action << 6) instead of the 4-B one
 *   skel-12     (mode 3) the skeleton's three 4-B results only (no partition entry)
 *   skel-8+1    (mode 4) the packed result layout's writes: one 8-B result (o0 holds n x 8 B) and the 1-B entry
 *   copy        a 16-B-per-lane copy, 4 loads in flight per lane (the guide's float4 copy, MI355X_MICROARCH.md:
 *               6.29 TB/s)
 *
 * Each launch also measures the shader clock it ran at: wave 0 of workgroup 0 (resident for the whole persistent
 * launch) reads the shader-clock counter (s_memtime) and the 100-MHz real-time counter (s_memrealtime) at its start
 * and end, so sclk = d(memtime) / d(memrealtime) x 100 MHz over the launch.
 */
#include <hip/hip_runtime.h>
#include <hip/hip_ext.h>

#include <stdint.h>

#define PPE_CALIB_MAXB 32

struct ppe_calib_batch {
    const uint8_t *hdr;
    const uint32_t *len;
    uint32_t *o0, *o1, *o2, *o3;
    uint32_t n, pad;
};
struct ppe_calib_args {
    ppe_calib_batch b[PPE_CALIB_MAXB];
    uint32_t nb, mode;
    unsigned long long *clk;  // [4]: memtime start / end, memrealtime start / end (wave 0 of workgroup 0)
};

namespace {

typedef uint32_t v4u __attribute__((ext_vector_type(4)));

__device__ __forceinline__ void clk_mark(const ppe_calib_args &a, int k) {
    if (a.clk && blockIdx.x == 0 && threadIdx.x == 0) {
        const unsigned long long t = __builtin_amdgcn_s_memtime(), r = __builtin_amdgcn_s_memrealtime();
        a.clk[k] = t;
        a.clk[2 + k] = r;
    }
}

// wave w of W takes global tiles w, w + W, ... over the batches in order (batch = tile / tiles-per-batch)
template <int MODE>
__global__ __launch_bounds__(512) void calib_kernel(ppe_calib_args a) {
    clk_mark(a, 0);
    const uint32_t lane = threadIdx.x & 63u;
    const uint32_t W = gridDim.x * 8u, w0 = blockIdx.x * 8u + (threadIdx.x >> 6);
    uint32_t acc = 0;
    for (uint32_t bi = 0; bi < a.nb; ++bi) {
        const ppe_calib_batch &B = a.b[bi];
        const uint32_t ntiles = (B.n + 63u) >> 6;
        for (uint32_t t = w0; t < ntiles; t += W) {
            const uint32_t p = min((t << 6) + lane, B.n - 1u);
            const v4u *r = (const v4u *)(B.hdr + (size_t)p * 64u);
            const v4u q0 = r[0], q1 = r[1], q2 = r[2];
            const uint32_t q3 = *(const uint32_t *)(r + 3);
            const uint32_t l = B.len[p];
            const uint32_t x = q0.x ^ q0.y ^ q0.z ^ q0.w ^ q1.x ^ q1.y ^ q1.z ^ q1.w ^ q2.x ^ q2.y ^ q2.z ^ q2.w ^ q3;
            if (MODE == 4) {
                if ((t << 6) + lane < B.n) {
                    typedef uint32_t v2u __attribute__((ext_vector_type(2)));
                    v2u r2;
                    r2.x = x;
                    r2.y = x ^ l;
                    __builtin_nontemporal_store(r2, (v2u *)B.o0 + p);
                    __builtin_nontemporal_store((uint8_t)((p & 63u) | ((x & 3u) << 6)), (uint8_t *)B.o3 + p);
                }
            } else if (MODE == 0 || MODE == 2 || MODE == 3) {
                if ((t << 6) + lane < B.n) {
                    __builtin_nontemporal_store(x, B.o0 + p);
                    __builtin_nontemporal_store(x ^ l, B.o1 + p);
                    __builtin_nontemporal_store(x + l, B.o2 + p);
                    if (MODE == 0) __builtin_nontemporal_store(p, B.o3 + p);
                    if (MODE == 2) __builtin_nontemporal_store((uint8_t)((p & 63u) | ((x & 3u) << 6)), (uint8_t *)B.o3 + p);
                }
            } else {
                acc ^= x + l;
            }
        }
        if (MODE == 1) {
            // one word per wave and batch (negligible traffic; keeps the loads live)
#pragma unroll
            for (int o = 32; o > 0; o >>= 1) acc ^= __shfl_xor(acc, o, 64);
            if (lane == 0 && w0 < ((B.n + 63u) >> 6)) B.o0[w0] = acc;
        }
    }
    // (the clock mark waits for wave 0's own loads; the launch's end timestamp is the dispatch's)
    clk_mark(a, 1);
}

// 4 independent 16-B loads in flight per lane before their stores (a one-load loop keeps too few bytes in flight
// per CU to reach the HBM rate: 5.1-5.2 TB/s measured in gpurun_out/r3b)
__global__ __launch_bounds__(512) void copy_kernel(const v4u *__restrict__ src, v4u *__restrict__ dst, size_t n16,
                                                   unsigned long long *clk) {
    if (clk && blockIdx.x == 0 && threadIdx.x == 0) {
        clk[0] = __builtin_amdgcn_s_memtime();
        clk[2] = __builtin_amdgcn_s_memrealtime();
    }
    const size_t stride = (size_t)gridDim.x * 512u;
    size_t i = (size_t)blockIdx.x * 512u + threadIdx.x;
    for (; i + 3u * stride < n16; i += 4u * stride) {
        const v4u a = __builtin_nontemporal_load(src + i), b = __builtin_nontemporal_load(src + i + stride),
                  c = __builtin_nontemporal_load(src + i + 2u * stride), d = __builtin_nontemporal_load(src + i + 3u * stride);
        __builtin_nontemporal_store(a, dst + i);
        __builtin_nontemporal_store(b, dst + i + stride);
        __builtin_nontemporal_store(c, dst + i + 2u * stride);
        __builtin_nontemporal_store(d, dst + i + 3u * stride);
    }
    for (; i < n16; i += stride) dst[i] = src[i];
    if (clk && blockIdx.x == 0 && threadIdx.x == 0) {
        clk[1] = __builtin_amdgcn_s_memtime();
        clk[3] = __builtin_amdgcn_s_memrealtime();
    }
}

}  // namespace

static int timed(hipStream_t s, double *ms_out, hipEvent_t *e) {
    if (hipEventSynchronize(e[1]) != hipSuccess) return (int)hipErrorUnknown;
    float ms = 0.f;
    const hipError_t r = hipEventElapsedTime(&ms, e[0], e[1]);
    if (ms_out) *ms_out = ms;
    (void)s;
    return (int)r;
}

static uint32_t default_grid(uint32_t grid) {
    if (grid) return grid;
    int dev = 0, ncu = 256;
    if (hipGetDevice(&dev) == hipSuccess) (void)hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev);
    return (uint32_t)ncu * 4u;  // 4 x 512 threads: 32 waves per CU, the classify kernel's C1 occupancy
}

extern "C" {

// mode 0 skeleton, 1 read-only, 2 skeleton with a 1-B partition entry, 3 skeleton without it, 4 the packed layout's
// 8 + 1 B.  grid = workgroups of 512 threads (persistent).  Returns a hipError_t.
int ppe_calib_stream(const ppe_calib_args *a, uint32_t grid, void *stream, void *ev0, void *ev1) {
    if (!a || a->nb == 0 || a->nb > PPE_CALIB_MAXB) return (int)hipErrorInvalidValue;
    for (uint32_t i = 0; i < a->nb; ++i)
        if (!a->b[i].hdr || !a->b[i].len || !a->b[i].o0 || a->b[i].n == 0 || (a->mode != 1 && !a->b[i].o3) ||
            ((a->mode == 0 || a->mode == 2 || a->mode == 3) && (!a->b[i].o1 || !a->b[i].o2)))
            return (int)hipErrorInvalidValue;
    if (a->mode == 0)
        hipExtLaunchKernelGGL(calib_kernel<0>, dim3(grid), dim3(512), 0, (hipStream_t)stream, (hipEvent_t)ev0,
                              (hipEvent_t)ev1, 0, *a);
    else if (a->mode == 2)
        hipExtLaunchKernelGGL(calib_kernel<2>, dim3(grid), dim3(512), 0, (hipStream_t)stream, (hipEvent_t)ev0,
                              (hipEvent_t)ev1, 0, *a);
    else if (a->mode == 4)
        hipExtLaunchKernelGGL(calib_kernel<4>, dim3(grid), dim3(512), 0, (hipStream_t)stream, (hipEvent_t)ev0,
                              (hipEvent_t)ev1, 0, *a);
    else if (a->mode == 3)
        hipExtLaunchKernelGGL(calib_kernel<3>, dim3(grid), dim3(512), 0, (hipStream_t)stream, (hipEvent_t)ev0,
                              (hipEvent_t)ev1, 0, *a);
    else
        hipExtLaunchKernelGGL(calib_kernel<1>, dim3(grid), dim3(512), 0, (hipStream_t)stream, (hipEvent_t)ev0,
                              (hipEvent_t)ev1, 0, *a);
    return (int)hipGetLastError();
}

// dst[i] = src[i] over `bytes` (a multiple of 16, 16-B aligned pointers)
int ppe_calib_copy(const void *src, void *dst, size_t bytes, uint32_t grid, unsigned long long *clk, void *stream,
                   void *ev0, void *ev1) {
    if (!src || !dst || (bytes & 15u) || (((uintptr_t)src | (uintptr_t)dst) & 15u)) return (int)hipErrorInvalidValue;
    hipExtLaunchKernelGGL(copy_kernel, dim3(grid), dim3(512), 0, (hipStream_t)stream, (hipEvent_t)ev0,
                          (hipEvent_t)ev1, 0, (const v4u *)src, (v4u *)dst, bytes / 16u, clk);
    return (int)hipGetLastError();
}


// Synchronous forms for bench.py: one launch with its dispatch timestamps, kernel milliseconds in *ms_out.
// grid 0 = 4 workgroups of 512 threads per CU.
int ppe_calib_stream_timed(const ppe_calib_args *a, uint32_t grid, void *stream, double *ms_out) {
    hipEvent_t e[2];
    if (hipEventCreate(&e[0]) != hipSuccess || hipEventCreate(&e[1]) != hipSuccess) return (int)hipErrorUnknown;
    int rc = ppe_calib_stream(a, default_grid(grid), stream, e[0], e[1]);
    if (rc == 0) rc = timed((hipStream_t)stream, ms_out, e);
    (void)hipEventDestroy(e[0]);
    (void)hipEventDestroy(e[1]);
    return rc;
}

int ppe_calib_copy_timed(const void *src, void *dst, size_t bytes, uint32_t grid, unsigned long long *clk,
                         void *stream, double *ms_out) {
    hipEvent_t e[2];
    if (hipEventCreate(&e[0]) != hipSuccess || hipEventCreate(&e[1]) != hipSuccess) return (int)hipErrorUnknown;
    int rc = ppe_calib_copy(src, dst, bytes, default_grid(grid), clk, stream, e[0], e[1]);
    if (rc == 0) rc = timed((hipStream_t)stream, ms_out, e);
    (void)hipEventDestroy(e[0]);
    (void)hipEventDestroy(e[1]);
    return rc;
}

}
