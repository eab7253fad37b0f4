// hh_probe.hip -- the streaming-copy reference bench.py divides by
// (frac_vs_copy): how fast a plain HBM stream runs on this GPU, measured on
// the same box in the same run as the decode.  Not on the decode path.
//
// One 16-B load and one 16-B store per lane, one element per lane: a grid of
// n / 256 workgroups of 256 and no grid-stride loop, loads and stores with
// the cache policy given (0 plain, 2 nt).  tools/ubench/ub_copy.hip swept the
// alternatives on 1.5 GB (bench.py's byte count): this shape 6.54 TB/s
// (read + write) nontemporal; grid-stride loops with 1..8 elements in flight
// per lane and 2..16 workgroups of 256..1024 per CU 4.7-5.9 TB/s.
#include <hip/hip_runtime.h>

#include <stdint.h>

#include "hiphuff.h"

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

#define CP_TB 256

template <int CPOL>
__global__ __launch_bounds__(CP_TB) void k_copy16(const u32x4 *__restrict__ src, u32x4 *__restrict__ dst, uint64_t n) {
    const uint64_t i = (uint64_t)blockIdx.x * CP_TB + threadIdx.x;
    if (i >= n) return;
    const u32x4 v = CPOL ? __builtin_nontemporal_load(src + i) : src[i];
    if (CPOL) __builtin_nontemporal_store(v, dst + i);
    else dst[i] = v;
}

// nbytes: a multiple of 16, both pointers 16-B aligned.  *ms: device time of
// the copy (HIP events on the stream).  Returns when done.
extern "C" int hh_copy_device(const void *d_src, void *d_dst, uint64_t nbytes, int nt, void *hip_stream, float *ms) {
    if (!d_src || !d_dst || !ms || nbytes % 16 || ((uintptr_t)d_src | (uintptr_t)d_dst) & 15u) return HH_ERR_ARG;
    hipStream_t st = (hipStream_t)hip_stream;
    const uint64_t n = nbytes / 16;
    const uint64_t blocks = (n + CP_TB - 1) / CP_TB;
    if (blocks > 0x7fffffffull) return HH_ERR_ARG;   // (a grid dimension's limit: 32 TiB)
    const unsigned grid = (unsigned)(blocks ? blocks : 1);
    hipEvent_t e0, e1;
    if (hipEventCreate(&e0) != hipSuccess) return HH_ERR_DEVICE;
    if (hipEventCreate(&e1) != hipSuccess) { (void)hipEventDestroy(e0); return HH_ERR_DEVICE; }
    int rc = HH_ERR_DEVICE;
    do {
        if (hipEventRecord(e0, st) != hipSuccess) break;
        if (nt) hipLaunchKernelGGL(k_copy16<2>, dim3(grid), dim3(CP_TB), 0, st, (const u32x4 *)d_src, (u32x4 *)d_dst, n);
        else hipLaunchKernelGGL(k_copy16<0>, dim3(grid), dim3(CP_TB), 0, st, (const u32x4 *)d_src, (u32x4 *)d_dst, n);
        if (hipGetLastError() != hipSuccess) break;
        if (hipEventRecord(e1, st) != hipSuccess || hipEventSynchronize(e1) != hipSuccess) break;
        if (hipEventElapsedTime(ms, e0, e1) != hipSuccess) break;
        rc = HH_OK;
    } while (0);
    (void)hipEventDestroy(e0);
    (void)hipEventDestroy(e1);
    return rc;
}
