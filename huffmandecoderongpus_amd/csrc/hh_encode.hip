// Device encoder: symbols (u8, in HBM) -> the LSB-first .huff bitstream of a
// code tree, the inverse of the decode path.  The reference ships no encoder
// (fast generation and round-trip checks of
// multi-GiB inputs); the bit order is the one its decoders read
// (framework/huffdata.c:55-64, decodeallbits.cl:23: stream bit p is bit
// p % 8 of byte p / 8) and the one hh_encode (csrc/hh_huff.c) writes on the
// host.  Three launches on the caller's stream:
//   k_enc_len   one workgroup per chunk of ENC_CH symbols: the chunk's code
//               bits (and whether a symbol is absent from the tree);
//   k_enc_scan  one workgroup: exclusive scan of the chunks' bits -> each
//               chunk's first bit, the total;
//   k_enc_pack  one workgroup per chunk: each thread's 16 symbols' codes
//               ORed into the chunk's image in LDS (aligned to the output's
//               32-bit words), then written out -- plain stores inside the
//               chunk, atomic ORs on its first and last word (shared with
//               the neighbouring chunks; the output is zeroed first).
// HBM-bound: 1 B read per symbol, its code bits written once.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdlib.h>

#include <mutex>

#include "hiphuff.h"
#include "hh_internal.h"

#define ENC_TB 256                 // threads per workgroup
#define ENC_PT 16                  // symbols per thread
#define ENC_CH (ENC_TB * ENC_PT)   // symbols per chunk
#define ENC_SCAN_TB 1024

// (lengths: u32 per symbol, 0 = absent; codes: u64, the first stream bit in
// bit 0)
struct EncTab {
    uint64_t code[256];
    uint32_t len[256];
};

__device__ __forceinline__ uint32_t enc_block_sum(uint32_t v, uint32_t *s_w) {
    const uint32_t tid = threadIdx.x, lane = tid & 63u, wv = tid >> 6;
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    if (lane == 0) s_w[wv] = v;
    __syncthreads();
    uint32_t t = 0;
#pragma unroll
    for (uint32_t i = 0; i < ENC_TB / 64; i++) t += s_w[i];
    return t;
}

// A thread's ENC_PT symbols from i0: one 16-B load when they are all in the
// stream and 16-B aligned (torch tensors are), else byte by byte.
__device__ __forceinline__ void enc_load16(const uint8_t *__restrict__ syms, uint64_t n, uint64_t i0, uint8_t *sy) {
    if (i0 + ENC_PT <= n && (((uintptr_t)(syms + i0)) & 15u) == 0) {
        typedef uint32_t u4 __attribute__((ext_vector_type(4)));
        const u4 v = __builtin_nontemporal_load((const u4 *)(syms + i0));
#pragma unroll
        for (uint32_t k = 0; k < ENC_PT; k++) sy[k] = (uint8_t)(v[k >> 2] >> (8 * (k & 3)));
    } else {
#pragma unroll
        for (uint32_t k = 0; k < ENC_PT; k++) sy[k] = i0 + k < n ? syms[i0 + k] : 0u;
    }
}

__global__ __launch_bounds__(ENC_TB) void k_enc_len(const uint8_t *__restrict__ syms, uint64_t n,
                                                    const EncTab *__restrict__ tab, uint64_t *__restrict__ cbits,
                                                    uint32_t *__restrict__ bad) {
    __shared__ uint32_t s_len[256];
    __shared__ uint32_t s_w[ENC_TB / 64];
    const uint32_t tid = threadIdx.x;
    s_len[tid] = tab->len[tid];
    __syncthreads();
    const uint64_t i0 = (uint64_t)blockIdx.x * ENC_CH + (uint64_t)tid * ENC_PT;
    uint8_t sy[ENC_PT];
    enc_load16(syms, n, i0, sy);
    uint32_t sum = 0;
    bool miss = false;
#pragma unroll
    for (uint32_t k = 0; k < ENC_PT; k++)
        if (i0 + k < n) {
            const uint32_t l = s_len[sy[k]];
            sum += l;
            miss |= l == 0;
        }
    const uint32_t tot = enc_block_sum(sum, s_w);
    if (tid == 0) cbits[blockIdx.x] = tot;
    if (miss) atomicOr(bad, 1u);
}

// One workgroup: cbits -> exclusive chunk offsets (in place), res[0..1] the
// total bits.
__global__ __launch_bounds__(ENC_SCAN_TB) void k_enc_scan(uint64_t *__restrict__ cbits, uint64_t nch,
                                                          uint64_t *__restrict__ res) {
    __shared__ uint64_t s_w[ENC_SCAN_TB / 64];
    const uint32_t tid = threadIdx.x, lane = tid & 63u, wv = tid >> 6;
    uint64_t carry = 0;
    for (uint64_t b0 = 0; b0 < nch; b0 += ENC_SCAN_TB) {
        const uint64_t v = b0 + tid < nch ? cbits[b0 + tid] : 0;
        uint64_t x = v;
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
            const uint64_t y = __shfl_up(x, o, 64);
            if (lane >= (uint32_t)o) x += y;
        }
        if (lane == 63) s_w[wv] = x;
        __syncthreads();
        uint64_t base = 0, tot = 0;
        for (uint32_t i = 0; i < ENC_SCAN_TB / 64; i++) {
            base += i < wv ? s_w[i] : 0;
            tot += s_w[i];
        }
        if (b0 + tid < nch) cbits[b0 + tid] = carry + base + x - v;
        carry += tot;
        __syncthreads();
    }
    if (tid == 0) res[0] = carry;
}

// The chunk's image: (sh0 + its bits + 31) / 32 words, sh0 = its first
// bit's position in the output word it starts in.
#define ENC_IMG_WORDS ((31u + ENC_CH * 64u + 31u) / 32u + 1u)

__global__ __launch_bounds__(ENC_TB) void k_enc_pack(const uint8_t *__restrict__ syms, uint64_t n,
                                                     const EncTab *__restrict__ tab,
                                                     const uint64_t *__restrict__ coff, uint64_t total,
                                                     uint32_t *__restrict__ out) {
    extern __shared__ __align__(16) uint32_t s_img[];
    __shared__ uint64_t s_code[256];
    __shared__ uint32_t s_len[256];
    __shared__ uint32_t s_w[ENC_TB / 64];
    const uint32_t tid = threadIdx.x, lane = tid & 63u, wv = tid >> 6;
    s_code[tid] = tab->code[tid];
    s_len[tid] = tab->len[tid];
    // the chunk: its first bit and its bit count
    const uint64_t gb = coff[blockIdx.x];
    const uint64_t ge = blockIdx.x + 1 < gridDim.x ? coff[blockIdx.x + 1] : total;
    const uint32_t sh0 = (uint32_t)(gb & 31u);
    const uint32_t nw = (uint32_t)((sh0 + (ge - gb) + 31u) / 32u);
    for (uint32_t i = tid; i < nw; i += ENC_TB) s_img[i] = 0u;
    __syncthreads();
    // this thread's symbols and their bits
    const uint64_t i0 = (uint64_t)blockIdx.x * ENC_CH + (uint64_t)tid * ENC_PT;
    uint8_t sy[ENC_PT];
    enc_load16(syms, n, i0, sy);
    uint32_t sum = 0;
#pragma unroll
    for (uint32_t k = 0; k < ENC_PT; k++) sum += i0 + k < n ? s_len[sy[k]] : 0u;
    // exclusive scan of the threads' bits within the chunk
    uint32_t x = sum;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const uint32_t y = __shfl_up(x, o, 64);
        if (lane >= (uint32_t)o) x += y;
    }
    if (lane == 63) s_w[wv] = x;
    __syncthreads();
    uint32_t base = 0;
#pragma unroll
    for (uint32_t i = 0; i < ENC_TB / 64; i++) base += i < wv ? s_w[i] : 0u;
    uint32_t p = sh0 + base + x - sum;     // (bit position in the image)
    // each code's bits ORed into its (up to three) image words
#pragma unroll
    for (uint32_t k = 0; k < ENC_PT; k++) {
        if (i0 + k >= n) break;
        const uint32_t l = s_len[sy[k]];
        const uint64_t c = s_code[sy[k]];
        const uint32_t w = p >> 5, o = p & 31u;
        const uint64_t v = c << o;
        if (l) atomicOr(&s_img[w], (uint32_t)v);
        if (o + l > 32u) atomicOr(&s_img[w + 1], (uint32_t)(v >> 32));
        if (o + l > 64u) atomicOr(&s_img[w + 2], (uint32_t)(c >> (64u - o)));
        p += l;
    }
    __syncthreads();
    // out: the chunk's first and last word shared with its neighbours
    uint32_t *dst = out + (gb >> 5);
    for (uint32_t i = tid; i < nw; i += ENC_TB) {
        if (i == 0 || i + 1 == nw) atomicOr(dst + i, s_img[i]);
        else dst[i] = s_img[i];
    }
}

// An encoder: the workspace of one device's encodes (the table, the chunks'
// bits / offsets, the total and the absent-symbol flag), kept across calls
// and grown when a call needs more.  Calls on one encoder run one at a time
// (each returns when its encode is done); encoders are independent, so
// encodes on several streams run at once with one encoder each.
struct hh_encoder {
    int device;
    uint8_t *ws;
    size_t size;
};

extern "C" int hh_encoder_create(hh_encoder **enc, int device) {
    if (!enc) return HH_ERR_ARG;
    *enc = nullptr;
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || device < 0 || device >= ndev) return HH_ERR_ARG;
    hh_encoder *e = (hh_encoder *)calloc(1, sizeof(hh_encoder));
    if (!e) return HH_ERR_NOMEM;
    e->device = device;
    *enc = e;
    return HH_OK;
}

extern "C" void hh_encoder_destroy(hh_encoder *enc) {
    if (!enc) return;
    if (enc->ws) {
        (void)hipSetDevice(enc->device);
        (void)hipFree(enc->ws);                        // (every encode on it has returned: nothing in flight)
    }
    free(enc);
}

extern "C" int hh_encoder_encode(hh_encoder *enc, const hh_tree *tree, const void *d_syms, uint64_t n, void *d_out,
                                 uint64_t cap, uint64_t *bits, void *hip_stream) {
    if (!enc || !tree || !bits || (!d_syms && n) || (!d_out && cap)) return HH_ERR_ARG;
    if (((uintptr_t)d_out & 3u) != 0) return HH_ERR_ARG;   // (32-bit word stores)
    *bits = 0;
    EncTab h;
    uint8_t len8[256];
    int rc = hh_codebook(tree, h.code, len8);
    if (rc) return rc;
    for (int i = 0; i < 256; i++) h.len[i] = len8[i];
    if (n == 0) return HH_OK;
    if (hipSetDevice(enc->device) != hipSuccess) return HH_ERR_DEVICE;
    hipStream_t st = (hipStream_t)hip_stream;
    const uint64_t nch = (n + ENC_CH - 1) / ENC_CH;
    // (a launch's grid may not exceed 2^32 - 1 threads: about 2^24 chunks,
    // 68.7 G symbols, with ENC_TB threads each)
    if (nch * ENC_TB > 0xffffffffull) return HH_ERR_UNSUPPORTED;
    const size_t o_cb = (sizeof(EncTab) + 255) & ~(size_t)255, o_res = o_cb + ((nch * 8 + 255) & ~(size_t)255);
    if (enc->size < o_res + 64) {
        // (the previous encode on this encoder has returned: its stream is
        // done with the old workspace, no device-wide wait)
        if (enc->ws) (void)hipFree(enc->ws);
        enc->ws = nullptr;
        enc->size = 0;
        if (hipMalloc(&enc->ws, o_res + 64) != hipSuccess) return HH_ERR_NOMEM;
        enc->size = o_res + 64;
    }
    uint8_t *ws = enc->ws;
    EncTab *d_tab = (EncTab *)ws;
    uint64_t *d_cb = (uint64_t *)(ws + o_cb), *d_res = (uint64_t *)(ws + o_res);
    uint32_t *d_bad = (uint32_t *)(ws + o_res + 32);
    uint64_t hres[5] = {0, 0, 0, 0, 0};
    rc = HH_ERR_DEVICE;
    do {
        if (hipMemcpyAsync(d_tab, &h, sizeof(h), hipMemcpyHostToDevice, st) != hipSuccess) break;
        if (hipMemsetAsync(ws + o_res, 0, 64, st) != hipSuccess) break;
        hipLaunchKernelGGL(k_enc_len, dim3((unsigned)nch), dim3(ENC_TB), 0, st, (const uint8_t *)d_syms, n, d_tab, d_cb,
                           d_bad);
        if (hipGetLastError() != hipSuccess) break;
        hipLaunchKernelGGL(k_enc_scan, dim3(1), dim3(ENC_SCAN_TB), 0, st, d_cb, nch, d_res);
        if (hipGetLastError() != hipSuccess) break;
        if (hipMemcpyAsync(hres, d_res, 40, hipMemcpyDeviceToHost, st) != hipSuccess) break;
        if (hipStreamSynchronize(st) != hipSuccess) break;
        if ((uint32_t)hres[4]) { rc = HH_ERR_ARG; break; }   // (a symbol absent from the tree)
        const uint64_t total = hres[0];
        *bits = total;
        const uint64_t need = (total + 31) / 32 * 4;            // (whole output words)
        if (need > cap) { rc = HH_ERR_CAPACITY; break; }
        if (hipMemsetAsync(d_out, 0, need, st) != hipSuccess) break;
        hipLaunchKernelGGL(k_enc_pack, dim3((unsigned)nch), dim3(ENC_TB), ENC_IMG_WORDS * 4, st,
                           (const uint8_t *)d_syms, n, d_tab, d_cb, total, (uint32_t *)d_out);
        if (hipGetLastError() != hipSuccess) break;
        if (hipStreamSynchronize(st) != hipSuccess) break;
        rc = HH_OK;
    } while (0);
    return rc;
}

// The handle-free form: one encoder per device for the process, calls
// serialised on it.
extern "C" int hh_encode_device(const hh_tree *tree, const void *d_syms, uint64_t n, void *d_out, uint64_t cap,
                                uint64_t *bits, void *hip_stream) {
    static std::mutex mu;
    static hh_encoder *s_enc[64];
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return HH_ERR_DEVICE;
    std::lock_guard<std::mutex> lock(mu);
    if (!s_enc[dev]) {
        const int rc = hh_encoder_create(&s_enc[dev], dev);
        if (rc) return rc;
    }
    return hh_encoder_encode(s_enc[dev], tree, d_syms, n, d_out, cap, bits, hip_stream);
}
