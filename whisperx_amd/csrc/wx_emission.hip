// wx_emission.hip — gfx950 kernels of the emission producer (reference
// whisperx/alignment.py:226-233, the wav2vec2 forward): the first feature-encoder layer's
// GroupNorm(512 groups = per channel over time) + GELU, fused, on time-major activations.
//
// emission.prepare_model keeps the conv feature encoder time-major ([L, C], the GEMM route's
// natural output).  torch's GroupNorm wants channel-major input, so on that layout it first
// copied the 96k x 512 activation (196 MB for a 30 s segment) and then normalised it: ~1 ms per
// forward.  Here: pass 1 reduces per-channel sums over time (column tiles, coalesced 256-B row
// segments, fp64 partials), pass 2 normalises, applies the affine and the exact (erf) GELU in
// one read + one write.  HBM-bound: ~3 x 4 B x L x C moved.
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdint.h>

#include "../../include/wx_align.h"

namespace wxe {

constexpr int kCols = 64;    // channels per column tile (one wave-row of 64 lanes: 256 B)
constexpr int kRows = 4;     // waves per block, each striding rows
constexpr int kSplit = 256;  // row slices per channel tile in pass 1

// pass 1: partial (sum, sum of squares) per (row slice, channel) in fp64
__global__ __launch_bounds__(kCols * kRows) void chan_stats_kernel(const float* __restrict__ x, int64_t L, int C,
                                                                  double* __restrict__ part /* [kSplit][2][C] */) {
    const int c = blockIdx.x * kCols + (threadIdx.x & (kCols - 1));
    const int r0 = threadIdx.x / kCols;
    const int slice = blockIdx.y;
    const int64_t per = (L + kSplit - 1) / kSplit;
    const int64_t lo = slice * per, hi = min(L, lo + per);
    double s = 0.0, q = 0.0;
    if (c < C) {
        for (int64_t t = lo + r0; t < hi; t += kRows) {
            const double v = (double)x[t * C + c];
            s += v;
            q += v * v;
        }
    }
    __shared__ double ss[kRows][kCols], qq[kRows][kCols];
    ss[r0][threadIdx.x & (kCols - 1)] = s;
    qq[r0][threadIdx.x & (kCols - 1)] = q;
    __syncthreads();
    if (r0 == 0 && c < C) {
        for (int r = 1; r < kRows; ++r) {
            s += ss[r][threadIdx.x];
            q += qq[r][threadIdx.x];
        }
        part[(int64_t)slice * 2 * C + c] = s;
        part[(int64_t)slice * 2 * C + C + c] = q;
    }
}

// mean / rstd per channel from the partials, folded with the affine: y = x * a + b
__global__ void chan_finish_kernel(const double* __restrict__ part, int64_t L, int C, const float* __restrict__ gamma,
                                   const float* __restrict__ beta, float eps, float* __restrict__ ab /* [2][C] */) {
    const int c = blockIdx.x * blockDim.x + threadIdx.x;
    if (c >= C) return;
    double s = 0.0, q = 0.0;
    for (int k = 0; k < kSplit; ++k) {
        s += part[(int64_t)k * 2 * C + c];
        q += part[(int64_t)k * 2 * C + C + c];
    }
    const double mean = s / (double)L;
    const double var = fmax(q / (double)L - mean * mean, 0.0);  // biased, as GroupNorm
    const double rstd = 1.0 / sqrt(var + (double)eps);
    const double g = gamma ? (double)gamma[c] : 1.0, b = beta ? (double)beta[c] : 0.0;
    ab[c] = (float)(rstd * g);
    ab[C + c] = (float)(b - mean * rstd * g);
}

__device__ __forceinline__ float gelu_erf(float v) { return 0.5f * v * (1.0f + erff(v * 0.70710678118654752f)); }

// pass 2: y = gelu(x * a[c] + b[c]), float4 per thread along channels
__global__ __launch_bounds__(256) void chan_apply_kernel(const float* __restrict__ x, int64_t n4, int C4,
                                                          const float* __restrict__ ab, int C, int gelu,
                                                          float* __restrict__ y) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n4) return;
    const int c = (int)(i % C4) * 4;
    const float4 v = reinterpret_cast<const float4*>(x)[i];
    float o[4] = {v.x * ab[c] + ab[C + c], v.y * ab[c + 1] + ab[C + c + 1], v.z * ab[c + 2] + ab[C + c + 2],
                  v.w * ab[c + 3] + ab[C + c + 3]};
    if (gelu) {
#pragma unroll
        for (int k = 0; k < 4; ++k) o[k] = gelu_erf(o[k]);
    }
    reinterpret_cast<float4*>(y)[i] = make_float4(o[0], o[1], o[2], o[3]);
}

// ------------------------------------------------------------------------------------
// The feature encoder's first layer as one pass over its output: conv (1 input channel, k taps,
// stride s: wav2vec2's 512 x 10 / 5) -> GroupNorm(one group per channel, over time) -> exact
// GELU, time-major [Lout, C].  Through the GEMM route this layer was a bias fill, a K = 10 GEMM
// writing 196 MB per 30 s segment (~12 TFLOP/s: HBM-bound on its own output), and the three
// channel-norm kernels reading it back twice (~230 us).  Here pass 1 computes the convolution in
// registers and reduces per-channel fp64 (sum, sum of squares) without writing it; pass 2
// recomputes it (k multiply-adds per value, cheaper than reading it back) and writes
// gelu(v * a[c] + b[c]) once.  A thread owns one channel (its k weights in registers) over
// kC0Rows consecutive rows; a wave covers 64 consecutive channels, so every row's store is 256
// contiguous bytes and the k waveform samples of a row are the same for the whole wave.
constexpr int kC0Rows = 16;  // rows per thread
constexpr int kC0MaxK = 16;  // taps held in registers

template <int K>
__device__ __forceinline__ float conv0_at(const float* __restrict__ x, int64_t t, int stride, const float (&w)[K],
                                          float bias) {
    const float* xr = x + t * stride;
    float v = bias;
#pragma unroll
    for (int j = 0; j < K; ++j) v = v + xr[j] * w[j];  // (-ffp-contract=off: separate multiply and add)
    return v;
}

template <int K>
__global__ __launch_bounds__(256) void conv0_stats_kernel(const float* __restrict__ x, int64_t L, int stride,
                                                          const float* __restrict__ wt, const float* __restrict__ bias,
                                                          int C, double* __restrict__ part /* [nblk][2][C] */) {
    const int c = blockIdx.x * kCols + (threadIdx.x & (kCols - 1));
    const int wv = threadIdx.x / kCols;
    float w[K];
#pragma unroll
    for (int j = 0; j < K; ++j) w[j] = c < C ? wt[(int64_t)c * K + j] : 0.f;
    const float b = (bias && c < C) ? bias[c] : 0.f;
    const int64_t t0 = ((int64_t)blockIdx.y * kRows + wv) * kC0Rows;
    double s = 0.0, q = 0.0;
    for (int r = 0; r < kC0Rows; ++r) {
        const int64_t t = t0 + r;
        if (t >= L) break;
        const double v = (double)conv0_at<K>(x, t, stride, w, b);
        s += v;
        q += v * v;
    }
    __shared__ double ss[kRows][kCols], qq[kRows][kCols];
    ss[wv][threadIdx.x & (kCols - 1)] = s;
    qq[wv][threadIdx.x & (kCols - 1)] = q;
    __syncthreads();
    if (wv == 0 && c < C) {
        for (int r = 1; r < kRows; ++r) {
            s += ss[r][threadIdx.x];
            q += qq[r][threadIdx.x];
        }
        part[(int64_t)blockIdx.y * 2 * C + c] = s;
        part[(int64_t)blockIdx.y * 2 * C + C + c] = q;
    }
}

// (a, b) per channel from nblk partials: 4 row groups per channel tile sum a quarter each with
// 8 loads in flight, combined in group order
__global__ __launch_bounds__(256) void conv0_finish_kernel(const double* __restrict__ part, int nblk, int64_t L, int C,
                                                           const float* __restrict__ gamma, const float* __restrict__ beta,
                                                           float eps, float* __restrict__ ab) {
    const int c = blockIdx.x * kCols + (threadIdx.x & (kCols - 1));
    const int g = threadIdx.x / kCols;
    double s = 0.0, q = 0.0;
    if (c < C) {
        const int lo = g * nblk / kRows, hi = (g + 1) * nblk / kRows;
        int k = lo;
        for (; k + 8 <= hi; k += 8) {
            double vs[8], vq[8];
#pragma unroll
            for (int u = 0; u < 8; ++u) {
                vs[u] = part[(int64_t)(k + u) * 2 * C + c];
                vq[u] = part[(int64_t)(k + u) * 2 * C + C + c];
            }
#pragma unroll
            for (int u = 0; u < 8; ++u) {
                s += vs[u];
                q += vq[u];
            }
        }
        for (; k < hi; ++k) {
            s += part[(int64_t)k * 2 * C + c];
            q += part[(int64_t)k * 2 * C + C + c];
        }
    }
    __shared__ double ss[kRows][kCols], qq[kRows][kCols];
    ss[g][threadIdx.x & (kCols - 1)] = s;
    qq[g][threadIdx.x & (kCols - 1)] = q;
    __syncthreads();
    if (g != 0 || c >= C) return;
    for (int r = 1; r < kRows; ++r) {
        s += ss[r][threadIdx.x];
        q += qq[r][threadIdx.x];
    }
    const double mean = s / (double)L;
    const double var = fmax(q / (double)L - mean * mean, 0.0);  // biased, as GroupNorm
    const double rstd = 1.0 / sqrt(var + (double)eps);
    const double gg = gamma ? (double)gamma[c] : 1.0, bb = beta ? (double)beta[c] : 0.0;
    ab[c] = (float)(rstd * gg);
    ab[C + c] = (float)(bb - mean * rstd * gg);
}

__device__ __forceinline__ float gelu_erf0(float v) { return 0.5f * v * (1.0f + erff(v * 0.70710678118654752f)); }

template <int K>
__global__ __launch_bounds__(256) void conv0_apply_kernel(const float* __restrict__ x, int64_t L, int stride,
                                                          const float* __restrict__ wt, const float* __restrict__ bias,
                                                          int C, const float* __restrict__ ab, int gelu,
                                                          float* __restrict__ y) {
    const int c = blockIdx.x * kCols + (threadIdx.x & (kCols - 1));
    const int wv = threadIdx.x / kCols;
    if (c >= C) return;
    float w[K];
#pragma unroll
    for (int j = 0; j < K; ++j) w[j] = wt[(int64_t)c * K + j];
    const float b = bias ? bias[c] : 0.f;
    const float sa = ab[c], sb = ab[C + c];
    const int64_t t0 = ((int64_t)blockIdx.y * kRows + wv) * kC0Rows;
#pragma unroll 4
    for (int r = 0; r < kC0Rows; ++r) {
        const int64_t t = t0 + r;
        if (t >= L) break;
        float v = conv0_at<K>(x, t, stride, w, b) * sa + sb;
        if (gelu) v = gelu_erf0(v);
        y[t * C + c] = v;
    }
}

// The same two passes for wav2vec2's geometry (K = 10 taps, stride 5), register-resident: a
// wave covers 32 consecutive rows x 64 channels, and the 165 waveform samples those rows read
// are loaded once (3 coalesced loads per lane) and broadcast per use with v_readlane (the
// sample index is uniform over the wave), instead of 10 dependent global loads per row
// (the generic kernels above: ~90 us per pass for a 30 s segment, latency-bound).  fma
// accumulation (equal to torch's conv to fp32 tolerance, like the generic path).
constexpr int kC0R = 32;  // rows per wave

template <int K, int S>
__device__ __forceinline__ float conv0_row(const float (&sv)[((kC0R - 1) * S + K + 63) / 64], int r, const float (&w)[K],
                                           float b) {
    float acc = b;
#pragma unroll
    for (int j = 0; j < K; ++j) {
        const int k = r * S + j;
        acc = fmaf(__int_as_float(__builtin_amdgcn_readlane(__float_as_int(sv[k >> 6]), k & 63)), w[j], acc);
    }
    return acc;
}

template <int K, int S>
__device__ __forceinline__ void conv0_samples(const float* __restrict__ x, int64_t nsamp, int64_t t0,
                                              float (&sv)[((kC0R - 1) * S + K + 63) / 64]) {
    constexpr int NV = ((kC0R - 1) * S + K + 63) / 64;
    const int l = threadIdx.x & 63;
#pragma unroll
    for (int v = 0; v < NV; ++v) {
        const int64_t i = t0 * S + 64 * v + l;
        sv[v] = i < nsamp ? x[i] : 0.f;
    }
}

// A wave whose kC0R rows read only samples inside the waveform (all but the last) reads them
// straight from memory at wave-uniform addresses: scalar loads into SGPRs that the FMAs take as
// operands — no v_readlane per tap and none of the SGPR-hazard s_nops after it (the register
// form, conv0_samples + conv0_row, stays for the last wave).  Same fma chain per row.
template <int K, int S>
__device__ __forceinline__ float conv0_row_s(const float* __restrict__ xs /* wave-uniform */, int r,
                                             const float (&w)[K], float b) {
    float acc = b;
#pragma unroll
    for (int j = 0; j < K; ++j) acc = fmaf(xs[r * S + j], w[j], acc);
    return acc;
}

template <int K, int S>
__global__ __launch_bounds__(256) void conv0_stats_rl_kernel(const float* __restrict__ x, int64_t nsamp, int64_t L,
                                                             const float* __restrict__ wt,
                                                             const float* __restrict__ bias, int C,
                                                             double* __restrict__ part /* [nblk][2][C] */) {
    const int lc = threadIdx.x & 63, wv = __builtin_amdgcn_readfirstlane((int)threadIdx.x >> 6);
    const int c = blockIdx.x * 64 + lc;
    const int cc = min(c, C - 1);
    float w[K];
#pragma unroll
    for (int j = 0; j < K; ++j) w[j] = wt[(int64_t)cc * K + j];
    const float b = bias ? bias[cc] : 0.f;
    const int64_t t0 = ((int64_t)blockIdx.y * 4 + wv) * kC0R;
    const int64_t nr = L - t0;
    double sm = 0.0, q = 0.0;
    if (t0 * S + (kC0R - 1) * S + K <= nsamp) {
        const float* xs = x + t0 * S;
#pragma unroll
        for (int r = 0; r < kC0R; ++r) {
            const double d = (double)conv0_row_s<K, S>(xs, r, w, b);
            if (r < nr) {
                sm += d;
                q = fma(d, d, q);
            }
        }
    } else {
        float sv[((kC0R - 1) * S + K + 63) / 64];
        conv0_samples<K, S>(x, nsamp, t0, sv);
#pragma unroll
        for (int r = 0; r < kC0R; ++r) {
            const double d = (double)conv0_row<K, S>(sv, r, w, b);
            if (r < nr) {
                sm += d;
                q = fma(d, d, q);
            }
        }
    }
    __shared__ double ss[4][64], qq[4][64];
    ss[wv][lc] = sm;
    qq[wv][lc] = q;
    __syncthreads();
    if (wv == 0 && c < C) {
        sm = (ss[0][lc] + ss[1][lc]) + (ss[2][lc] + ss[3][lc]);
        q = (qq[0][lc] + qq[1][lc]) + (qq[2][lc] + qq[3][lc]);
        part[(int64_t)blockIdx.y * 2 * C + c] = sm;
        part[(int64_t)blockIdx.y * 2 * C + C + c] = q;
    }
}

template <int K, int S>
__global__ __launch_bounds__(256) void conv0_apply_rl_kernel(const float* __restrict__ x, int64_t nsamp, int64_t L,
                                                             const float* __restrict__ wt,
                                                             const float* __restrict__ bias, int C,
                                                             const float* __restrict__ ab, int gelu,
                                                             float* __restrict__ y) {
    const int lc = threadIdx.x & 63, wv = __builtin_amdgcn_readfirstlane((int)threadIdx.x >> 6);
    const int c = blockIdx.x * 64 + lc;
    const int cc = min(c, C - 1);
    float w[K];
#pragma unroll
    for (int j = 0; j < K; ++j) w[j] = wt[(int64_t)cc * K + j];
    const float b = bias ? bias[cc] : 0.f;
    const float sa = ab[cc], sb = ab[C + cc];
    const int64_t t0 = ((int64_t)blockIdx.y * 4 + wv) * kC0R;
    const int64_t nr = L - t0;
    float* yr = y + t0 * C + c;  // (row r at yr + r C)
    if (t0 * S + (kC0R - 1) * S + K <= nsamp) {
        const float* xs = x + t0 * S;
#pragma unroll
        for (int r = 0; r < kC0R; ++r) {
            float v = conv0_row_s<K, S>(xs, r, w, b) * sa + sb;
            if (gelu) v = gelu_erf0(v);
            if (r < nr && c < C) yr[(int64_t)r * C] = v;
        }
    } else {
        float sv[((kC0R - 1) * S + K + 63) / 64];
        conv0_samples<K, S>(x, nsamp, t0, sv);
#pragma unroll
        for (int r = 0; r < kC0R; ++r) {
            float v = conv0_row<K, S>(sv, r, w, b) * sa + sb;
            if (gelu) v = gelu_erf0(v);
            if (r < nr && c < C) yr[(int64_t)r * C] = v;
        }
    }
}

// ------------------------------------------------------------------------------------
// wav2vec2 self-attention, fp32 (alignment.py:226-233: the encoder's 12 / 24 attention layers,
// one unpadded segment per forward, no mask).  torch's fused attention kernel for fp32
// (aotriton attn_fwd) took 34% of config 3's GPU time at ~26 TFLOP/s (profiles/
// r2_config3_kernel_stats.csv: 246 us per layer of a 29 s chunk).  Here: a flash-attention
// forward on the f32-input MFMA (v_mfma_f32_32x32x2_f32: exact f32 fmaf chains, 64 FLOP per
// clock per SIMD), one workgroup per (batch, head, 32-query tile) whose kAttnSplit waves take
// every kAttnSplit-th 32-key tile (a single 30 s segment has only 12 x 47 query tiles) and
// merge their (max, sum, O) states through LDS at the end; per wave:
//   * S^T = K Q^T per 32-key tile: lane l holds key row (l & 31) of K and query row (l & 31)
//     of Q as the A / B operands; the head dimension is split 32 / 32 between the lane halves
//     (the contraction order is free), so each lane reads contiguous 128-B half rows;
//   * S^T's accumulator has the query on the lane and 16 keys per lane in registers, so the
//     online softmax is lane-local plus one exchange with the other lane half, and the same
//     registers are the B operand (P^T) of O^T += V^T P^T without any lane movement: MFMA j
//     takes key (j & 3) + 8 (j >> 2) + 4 (l >> 5) from each half, and V is read at those rows;
//   * O^T lives in two 32x32 accumulators (head dims 0-31, 32-63), rescaled lane-locally.
// Not bit-identical to torch's kernel (different summation order); tests compare it with
// torch's attention at fp32 tolerance and the whole prepared forward with the stock one.
typedef float f32x16 __attribute__((ext_vector_type(16)));

struct AttnArgs {
    const float* q;
    const float* k;
    const float* v;
    float* o;  // [B, T, H, 64] (packed: [rows, H, 64])
    int B, H, T;
    int64_t sqb, sqh, sqt, skb, skh, skt, svb, svh, svt;  // element strides (head dim: 1)
    float scale_log2;                                      // softmax scale * log2(e)
    // packed segments (wx_attention_f32_packed): segment s owns rows [seg_rows[s], seg_rows[s+1])
    // and work units [seg_units[s], seg_units[s+1]) (H x its 32-query tiles, head-major)
    const int32_t* seg_rows;
    const int32_t* seg_units;
    int nseg;
};

constexpr int kAttnSplit = 4;  // waves per 32-query tile, each over every kAttnSplit-th 32-key tile

// amdgpu_waves_per_eu(2): two waves per SIMD, stated so the allocator keeps everything in VGPRs
// (~230 with the buffer-descriptor loads) instead of splitting them with AGPR copies (A/B: 1-2%
// faster).  A third wave per SIMD (168 registers: V loaded behind the S chain instead of a tile
// ahead, 2 spills) was 10-15% slower.  Round 6: the K / V loads through per-tile buffer
// descriptors (no per-lane address arithmetic) and no key compare on whole tiles took 12 packed
// 30 s segments (H = 12) from 818 to 727 us per call; PMC before the change: 327 VALU
// instructions per (wave, key tile) beside 64 MFMAs, ~150 of them address arithmetic (32-bit
// multiplies and 64-bit adds), MFMA busy 65% of the cycles.  With it the software-pipelined
// one-wave form of the same kernel (tile k + 1's S chain beside tile k's softmax, +2% before)
// measured equal (729 us) and was removed.
// SPLIT waves per 32-query tile (each over every SPLIT-th 32-key tile; SPLIT = 1: one wave, no
// merge); PACKED: one launch over many segments of their own lengths (rows packed back to back)
template <int SPLIT, bool PACKED>
__global__ __launch_bounds__(64 * SPLIT) __attribute__((amdgpu_waves_per_eu(2))) void attn_f32_kernel(AttnArgs a) {
    int T, tile, h;
    int64_t row0;  // o row of query 0 of this batch entry / segment
    const float *Q, *K, *V;
    // 1-D grid, block L runs on XCD L % 8 (round-robin dispatch): hand each XCD a contiguous
    // run of (head, query tile) units, so the blocks sharing one head's K / V (768 KB at
    // T = 1499) meet in one XCD's L2 instead of all eight
    // (round 4 A/B: the plain blockIdx order was 1-2% slower)
    const unsigned w = [] {
        const unsigned L = blockIdx.x, n = gridDim.x, x = L % 8, i = L / 8, q = n / 8, r = n % 8;
        return x * q + min(x, r) + i;
    }();
    if (PACKED) {
        // the segment owning unit w: the last s with seg_units[s] <= w (empty segments own no
        // units, so the last such s is never one of them)
        int lo = 0, hi = a.nseg - 1;
        while (lo < hi) {
            const int mid = (lo + hi + 1) >> 1;
            if ((unsigned)a.seg_units[mid] <= w) lo = mid;
            else hi = mid - 1;
        }
        row0 = a.seg_rows[lo];
        T = a.seg_rows[lo + 1] - (int)row0;
        const int nq = (T + 31) / 32;
        const int u = (int)w - a.seg_units[lo];
        tile = u % nq;
        h = u / nq;
        Q = a.q + row0 * a.sqt + h * a.sqh;
        K = a.k + row0 * a.skt + h * a.skh;
        V = a.v + row0 * a.svt + h * a.svh;
    } else {
        T = a.T;
        const int nq = (T + 31) / 32;
        tile = (int)(w % (unsigned)nq);
        const int bh = (int)(w / (unsigned)nq);
        const int b = bh / a.H;
        h = bh % a.H;
        row0 = (int64_t)b * T;
        Q = a.q + b * a.sqb + h * a.sqh;
        K = a.k + b * a.skb + h * a.skh;
        V = a.v + b * a.svb + h * a.svh;
    }
    const int q0 = tile * 32;
    const int l = threadIdx.x & 63, r = l & 31, hf = l >> 5, wv = threadIdx.x >> 6;
    float qv[32];
    {
        const float4* qp = reinterpret_cast<const float4*>(Q + (int64_t)min(q0 + r, T - 1) * a.sqt + 32 * hf);
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            const float4 x = qp[i];
            qv[4 * i] = x.x;
            qv[4 * i + 1] = x.y;
            qv[4 * i + 2] = x.z;
            qv[4 * i + 3] = x.w;
        }
    }
    f32x16 o0, o1;
#pragma unroll
    for (int i = 0; i < 16; ++i) o0[i] = o1[i] = 0.f;
    float m = -INFINITY, lsum = 0.f;
    // K / V of the wave's next key tile are loaded while the current one computes, through
    // buffer descriptors rebased per key tile (as attn_f32_pipe_kernel: no per-lane address
    // arithmetic; keys past the end read zeros, masked like the clamped re-reads they replace)
    float kv[32], va[16], vb[16];  // K[key r][32 hf + j]; V[key(j)][r], V[key(j)][32 + r]
    const int64_t skt = a.skt, svt = a.svt;
    const int vk = (int)((r * skt + 32 * hf) * 4), vv = (int)((4 * hf * svt + r) * 4);
    auto tile_rsrc = [&](const float* base, int64_t stride, int k0) {
        k0 = __builtin_amdgcn_readfirstlane(k0);  // (32 wv + ...: uniform, which hipcc cannot prove)
        const int64_t rem = (int64_t)(T - 1 - k0) * stride + 64;
        const int n = rem <= 0 ? 0 : (int)min(rem * 4, (int64_t)0x7fffffff);
        return __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(base + (int64_t)k0 * stride), 0, n, 0x00020000);
    };
    auto load_kv = [&](int k0, float(&kk)[32], float(&a0)[16], float(&a1)[16]) {
        typedef unsigned u4 __attribute__((ext_vector_type(4)));
        const __amdgpu_buffer_rsrc_t rk = tile_rsrc(K, skt, k0), rv = tile_rsrc(V, svt, k0);
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            const u4 x = __builtin_bit_cast(u4, __builtin_amdgcn_raw_buffer_load_b128(rk, vk + 16 * i, 0, 0));
            kk[4 * i] = __uint_as_float(x.x);
            kk[4 * i + 1] = __uint_as_float(x.y);
            kk[4 * i + 2] = __uint_as_float(x.z);
            kk[4 * i + 3] = __uint_as_float(x.w);
        }
#pragma unroll
        for (int j = 0; j < 16; ++j) {
            const int so = (int)(((j & 3) + 8 * (j >> 2)) * svt * 4);
            a0[j] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(rv, vv, so, 0));
            a1[j] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(rv, vv + 128, so, 0));
        }
    };
    if (32 * wv < T) load_kv(32 * wv, kv, va, vb);
    for (int k0 = 32 * wv; k0 < T; k0 += 32 * SPLIT) {
        f32x16 s;
#pragma unroll
        for (int i = 0; i < 16; ++i) s[i] = 0.f;
#pragma unroll
        for (int j = 0; j < 32; ++j) s = __builtin_amdgcn_mfma_f32_32x32x2f32(kv[j], qv[j], s, 0, 0, 0);
        float van[16], vbn[16];
        load_kv(k0 + 32 * SPLIT, kv, van, vbn);  // (past the end: zeros, unused); kv is dead once the S chain has been issued
        float mx = -INFINITY;
        if (k0 + 32 <= T) {  // a whole key tile: no key compare (uniform branch)
#pragma unroll
            for (int i = 0; i < 16; ++i) {
                s[i] = s[i] * a.scale_log2;
                mx = fmaxf(mx, s[i]);
            }
        } else {
#pragma unroll
            for (int i = 0; i < 16; ++i) {
                const int key = k0 + (i & 3) + 8 * (i >> 2) + 4 * hf;
                const float x = key < T ? s[i] * a.scale_log2 : -INFINITY;
                s[i] = x;
                mx = fmaxf(mx, x);
            }
        }
        mx = fmaxf(mx, __shfl_xor(mx, 32));
        const float mn = fmaxf(m, mx);
        const float alpha = __builtin_amdgcn_exp2f(m - mn);
        float ps = 0.f;
#pragma unroll
        for (int i = 0; i < 16; ++i) {
            const float p = __builtin_amdgcn_exp2f(s[i] - mn);
            s[i] = p;
            ps += p;
        }
        ps += __shfl_xor(ps, 32);
        lsum = lsum * alpha + ps;
        m = mn;
        if (__any(alpha != 1.0f)) {  // (the running maximum settles after a few tiles)
#pragma unroll
            for (int i = 0; i < 16; ++i) {
                o0[i] *= alpha;
                o1[i] *= alpha;
            }
        }
#pragma unroll
        for (int j = 0; j < 16; ++j) {
            o0 = __builtin_amdgcn_mfma_f32_32x32x2f32(va[j], s[j], o0, 0, 0, 0);
            o1 = __builtin_amdgcn_mfma_f32_32x32x2f32(vb[j], s[j], o1, 0, 0, 0);
        }
#pragma unroll
        for (int j = 0; j < 16; ++j) {
            va[j] = van[j];
            vb[j] = vbn[j];
        }
    }
    // merge the waves' partial softmax states (m, lsum, O^T) in wave 0
    if constexpr (SPLIT > 1) {
    __shared__ float red[SPLIT - 1][34][64];
    if (wv > 0) {
        float* o = &red[wv - 1][0][l];
        o[0] = m;
        o[64] = lsum;
#pragma unroll
        for (int i = 0; i < 16; ++i) {
            o[64 * (2 + i)] = o0[i];
            o[64 * (18 + i)] = o1[i];
        }
    }
    __syncthreads();
    if (wv > 0) return;
    float mt = m;
#pragma unroll
    for (int w = 0; w < SPLIT - 1; ++w) mt = fmaxf(mt, red[w][0][l]);
    {
        const float c = __builtin_amdgcn_exp2f(m - mt);
        lsum *= c;
#pragma unroll
        for (int i = 0; i < 16; ++i) {
            o0[i] *= c;
            o1[i] *= c;
        }
    }
#pragma unroll
    for (int w = 0; w < SPLIT - 1; ++w) {
        const float c = __builtin_amdgcn_exp2f(red[w][0][l] - mt);  // a wave without keys: 0
        lsum += red[w][1][l] * c;
#pragma unroll
        for (int i = 0; i < 16; ++i) {
            o0[i] += red[w][2 + i][l] * c;
            o1[i] += red[w][18 + i][l] * c;
        }
    }
    }
    if (q0 + r >= T) return;
    const float inv = 1.0f / lsum;
    float* orow = a.o + ((row0 + q0 + r) * a.H + h) * 64;
#pragma unroll
    for (int g = 0; g < 4; ++g) {  // registers 4g..4g+3: head dims 8g + 4hf + 0..3
        const int d = 8 * g + 4 * hf;
        *reinterpret_cast<float4*>(orow + d) =
            make_float4(o0[4 * g] * inv, o0[4 * g + 1] * inv, o0[4 * g + 2] * inv, o0[4 * g + 3] * inv);
        *reinterpret_cast<float4*>(orow + 32 + d) =
            make_float4(o1[4 * g] * inv, o1[4 * g + 1] * inv, o1[4 * g + 2] * inv, o1[4 * g + 3] * inv);
    }
}

// Residual add + LayerNorm over rows of D floats (the wav2vec2 encoder layer's
// `layer_norm(residual + x)`, twice per layer): one wave per row, the row in registers (D / 256
// float4 per lane), mean and biased variance in fp32 from the registers (two passes, not
// torch's Welford: equal to fp32 tolerance), y = (s - mean) * rstd * gamma + beta.  Optionally
// also writes the sum s (the pre-norm residual stream of the stable-layer-norm layers).
template <int NV>  // float4 per lane: D = 256 NV
__global__ __launch_bounds__(256) void add_ln_kernel(const float* __restrict__ a, const float* __restrict__ b,
                                                      const float* __restrict__ gamma, const float* __restrict__ beta,
                                                      float eps, int64_t rows, int64_t sa, int64_t sb, int64_t sy,
                                                      float* __restrict__ y, float* __restrict__ sum_out) {
    const int64_t row = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    if (row >= rows) return;
    const int l = threadIdx.x & 63;
    constexpr int D = 256 * NV;
    const float4* pa = reinterpret_cast<const float4*>(a + row * sa);
    const float4* pb = reinterpret_cast<const float4*>(b + row * sb);
    float4 v[NV];
    float acc = 0.0f;
#pragma unroll
    for (int i = 0; i < NV; ++i) {
        const float4 x = pa[64 * i + l], z = pb[64 * i + l];
        v[i] = make_float4(x.x + z.x, x.y + z.y, x.z + z.z, x.w + z.w);
        acc += (v[i].x + v[i].y) + (v[i].z + v[i].w);
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) acc += __shfl_xor(acc, o);
    const float mean = acc / (float)D;
    float q = 0.0f;
#pragma unroll
    for (int i = 0; i < NV; ++i) {
        const float dx = v[i].x - mean, dy = v[i].y - mean, dz = v[i].z - mean, dw = v[i].w - mean;
        q += (dx * dx + dy * dy) + (dz * dz + dw * dw);
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) q += __shfl_xor(q, o);
    const float rstd = 1.0f / sqrtf(q / (float)D + eps);
    float4* py = reinterpret_cast<float4*>(y + row * sy);
    float4* ps = sum_out ? reinterpret_cast<float4*>(sum_out + row * sy) : nullptr;
    const float4* pg = reinterpret_cast<const float4*>(gamma);
    const float4* pt = reinterpret_cast<const float4*>(beta);
#pragma unroll
    for (int i = 0; i < NV; ++i) {
        const float4 g = pg[64 * i + l], t = pt[64 * i + l];
        py[64 * i + l] = make_float4((v[i].x - mean) * rstd * g.x + t.x, (v[i].y - mean) * rstd * g.y + t.y,
                                     (v[i].z - mean) * rstd * g.z + t.z, (v[i].w - mean) * rstd * g.w + t.w);
        if (ps) ps[64 * i + l] = v[i];
    }
}

// ------------------------------------------------------------------------------------
// wav2vec2 positional convolution over packed segments (alignment.py:226-233: the encoder's
// Wav2Vec2PositionalConvEmbedding — Conv1d(D, D, K = 128, padding K / 2, groups G), the last
// output dropped, GELU — run per segment, zero padding at each segment's own ends).  As
// GEMMs it is G x [T, K Cg] x [K Cg, Cg] per segment with a patch operand (im2col of 128
// shifted rows) that torch had to gather, 4 x 32-tap blocks: 0.42 ms per 30 s segment at
// ~34 TFLOP/s.  Here one block per (segment, 128-frame tile, group): the tile's input window
// (255 rows x Cg channels) sits in LDS once and every tap reads its A fragments from it
// shifted by one row; the group's weights stream tap by tap through a double-buffered LDS
// slab (register-staged a tap ahead).  4 waves x 32 frames x Cg outputs on
// v_mfma_f32_16x16x4_f32 (exact f32 fma chains: not bit-identical to torch's conv, whose
// summation order differs); bias, erf GELU and optionally the residual (h + pos) fused.
constexpr int kPcFrames = 128;  // output frames per block (4 waves x 32)
constexpr int kPcK = 128;       // taps (wav2vec2's num_conv_pos_embeddings)
typedef float f32x4 __attribute__((ext_vector_type(4)));

struct PosConvArgs {
    const float* h;      // [rows, D] packed segments
    const float* w;      // [G][K][Cg / 4][Cg][4]: w[g][j][i / 4][o][i % 4] = conv.weight[g Cg + o][i][j]
    const float* bias;   // [D] or null
    float* out;          // [rows, D]
    const int32_t* seg_rows;
    const int32_t* seg_tiles;  // prefix of ceil(T_s / kPcFrames)
    int nseg, D;
    int residual;
};

template <int CG>
__global__ __launch_bounds__(256) void posconv_kernel(PosConvArgs a) {
    constexpr int RS = CG + 4;  // window row stride (floats): 16-B rows, banks spread over 16 rows
    constexpr int WR = kPcFrames + kPcK - 1;
    constexpr int NOB = CG / 16, NIC = CG / 16;
    constexpr int NB4 = CG * CG / 4;  // float4 per tap of the group's weights
    constexpr int PER = (NB4 + 255) / 256;
    __shared__ __attribute__((aligned(16))) float xa[WR * RS];
    __shared__ __attribute__((aligned(16))) float wb[2][CG * CG];
    const int g = blockIdx.y;
    const int w = blockIdx.x;
    int lo = 0, hi = a.nseg - 1;
    while (lo < hi) {
        const int mid = (lo + hi + 1) >> 1;
        if (a.seg_tiles[mid] <= w) lo = mid;
        else hi = mid - 1;
    }
    const int row0 = a.seg_rows[lo];
    const int T = a.seg_rows[lo + 1] - row0;
    const int t0 = (w - a.seg_tiles[lo]) * kPcFrames;
    const float* hg = a.h + (int64_t)row0 * a.D + g * CG;
    // the input window: row r <-> segment frame t0 - K / 2 + r (zero outside [0, T))
    for (int e = threadIdx.x; e < WR * (CG / 4); e += 256) {
        const int r = e / (CG / 4), c4 = e - r * (CG / 4);
        const int t = t0 - kPcK / 2 + r;
        float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
        if (t >= 0 && t < T) v = *reinterpret_cast<const float4*>(hg + (int64_t)t * a.D + 4 * c4);
        *reinterpret_cast<float4*>(xa + r * RS + 4 * c4) = v;
    }
    const float4* wg = reinterpret_cast<const float4*>(a.w) + (int64_t)g * kPcK * NB4;
    // the next tap's weights in named registers, loaded unconditionally (the last slot of a
    // partial tap re-reads a valid element, not stored) and pinned above the tap's MFMAs by a
    // sched_barrier: a register array with conditional stores had hipcc sink each load into
    // its store's branch after the MFMAs — a global round trip per slot and tap
    static_assert(PER <= 4, "posconv: at most four float4 slots per thread");
    float4 b0, b1, b2, b3;
    auto bload = [&](int j) {
        const float4* src = wg + (int64_t)j * NB4;
        const int t = (int)threadIdx.x;
        b0 = src[min(t, NB4 - 1)];
        if constexpr (PER > 1) b1 = src[min(t + 256, NB4 - 1)];
        if constexpr (PER > 2) b2 = src[min(t + 512, NB4 - 1)];
        if constexpr (PER > 3) b3 = src[min(t + 768, NB4 - 1)];
    };
    auto bstore = [&](int buf) {
        float4* dst = reinterpret_cast<float4*>(wb[buf]);
        const int t = (int)threadIdx.x;
        if (t < NB4) dst[t] = b0;
        if constexpr (PER > 1) if (t + 256 < NB4) dst[t + 256] = b1;
        if constexpr (PER > 2) if (t + 512 < NB4) dst[t + 512] = b2;
        if constexpr (PER > 3) if (t + 768 < NB4) dst[t + 768] = b3;
    };
    bload(0);
    bstore(0);
    __syncthreads();
    const int l = threadIdx.x & 63, wv = threadIdx.x >> 6, q = l >> 4, r16 = l & 15;
    f32x4 acc[2][NOB];
#pragma unroll
    for (int fb = 0; fb < 2; ++fb)
#pragma unroll
        for (int ob = 0; ob < NOB; ++ob) acc[fb][ob] = f32x4{0.f, 0.f, 0.f, 0.f};
    // A fragment rows: frame wv 32 + 16 fb + r16 of the tile, shifted by the tap
    const float* xrow = xa + (wv * 32 + r16) * RS + 4 * q;
    for (int j = 0; j < kPcK; ++j) {
        if (j + 1 < kPcK) bload(j + 1);
        __builtin_amdgcn_sched_barrier(0);
        const float* bb = wb[j & 1] + (q * CG + r16) * 4;
#pragma unroll
        for (int ic = 0; ic < NIC; ++ic) {
            float4 av[2], bv[NOB];
#pragma unroll
            for (int fb = 0; fb < 2; ++fb) av[fb] = *reinterpret_cast<const float4*>(xrow + (16 * fb + j) * RS + 16 * ic);
#pragma unroll
            for (int ob = 0; ob < NOB; ++ob) bv[ob] = *reinterpret_cast<const float4*>(bb + (ic * 4 * CG + 16 * ob) * 4);
#pragma unroll
            for (int fb = 0; fb < 2; ++fb)
#pragma unroll
                for (int ob = 0; ob < NOB; ++ob) {
                    acc[fb][ob] = __builtin_amdgcn_mfma_f32_16x16x4f32(av[fb].x, bv[ob].x, acc[fb][ob], 0, 0, 0);
                    acc[fb][ob] = __builtin_amdgcn_mfma_f32_16x16x4f32(av[fb].y, bv[ob].y, acc[fb][ob], 0, 0, 0);
                    acc[fb][ob] = __builtin_amdgcn_mfma_f32_16x16x4f32(av[fb].z, bv[ob].z, acc[fb][ob], 0, 0, 0);
                    acc[fb][ob] = __builtin_amdgcn_mfma_f32_16x16x4f32(av[fb].w, bv[ob].w, acc[fb][ob], 0, 0, 0);
                }
        }
        if (j + 1 < kPcK) bstore((j + 1) & 1);
        __syncthreads();
    }
    // accumulator (fb, ob) register v: frame 16 fb + 4 q + v of the wave's 32, output 16 ob + r16
#pragma unroll
    for (int fb = 0; fb < 2; ++fb)
#pragma unroll
        for (int v = 0; v < 4; ++v) {
            const int t = t0 + wv * 32 + 16 * fb + 4 * q + v;
            if (t >= T) continue;
            const int64_t rb = (int64_t)(row0 + t) * a.D + g * CG;
#pragma unroll
            for (int ob = 0; ob < NOB; ++ob) {
                const int c = 16 * ob + r16;
                float y = acc[fb][ob][v] + (a.bias ? a.bias[g * CG + c] : 0.f);
                y = gelu_erf0(y);
                if (a.residual) y += a.h[rb + c];
                a.out[rb + c] = y;
            }
        }
}

}  // namespace wxe

extern "C" size_t wx_channel_norm_workspace_bytes(int32_t C) {
    return (size_t)wxe::kSplit * 2 * C * sizeof(double) + 2 * (size_t)C * sizeof(float);
}

extern "C" int wx_channel_norm(const float* x, int64_t L, int32_t C, const float* gamma, const float* beta, float eps,
                               int32_t gelu, float* y, void* workspace, size_t workspace_bytes, void* stream) {
    using namespace wxe;
    if (L < 0 || C <= 0 || (C & 3) || !x || !y || !workspace) return WX_E_INVALID;
    if (workspace_bytes < wx_channel_norm_workspace_bytes(C)) return WX_E_WORKSPACE;
    if (L == 0) return WX_OK;
    if ((reinterpret_cast<uintptr_t>(x) & 15) || (reinterpret_cast<uintptr_t>(y) & 15)) return WX_E_INVALID;
    hipStream_t st = reinterpret_cast<hipStream_t>(stream);
    double* part = reinterpret_cast<double*>(workspace);
    float* ab = reinterpret_cast<float*>(part + (size_t)kSplit * 2 * C);
    hipLaunchKernelGGL(chan_stats_kernel, dim3((C + kCols - 1) / kCols, kSplit), dim3(kCols * kRows), 0, st, x, L, C,
                       part);
    hipLaunchKernelGGL(chan_finish_kernel, dim3((C + 255) / 256), dim3(256), 0, st, part, L, C, gamma, beta, eps, ab);
    const int64_t n4 = L * (C / 4);
    hipLaunchKernelGGL(chan_apply_kernel, dim3((unsigned)((n4 + 255) / 256)), dim3(256), 0, st, x, n4, C / 4, ab, C,
                       gelu, y);
    const hipError_t e = hipGetLastError();
    return e == hipSuccess ? WX_OK : (int)e;
}

extern "C" size_t wx_conv0_channel_norm_workspace_bytes(int64_t L, int32_t C) {
    if (L <= 0 || C <= 0) return 0;
    const int64_t nblk = (L + wxe::kRows * wxe::kC0Rows - 1) / (wxe::kRows * wxe::kC0Rows);
    return (size_t)nblk * 2 * C * sizeof(double) + 2 * (size_t)C * sizeof(float);
}

extern "C" int wx_conv0_channel_norm(const float* x, int64_t S, int32_t K, int32_t stride, const float* w,
                                     const float* bias, int32_t C, const float* gamma, const float* beta, float eps,
                                     int32_t gelu, float* y, void* workspace, size_t workspace_bytes, void* stream) {
    using namespace wxe;
    if (S < 0 || C <= 0 || K < 1 || K > kC0MaxK || stride < 1 || !x || !w || !y) return WX_E_INVALID;
    const int64_t L = S >= K ? (S - K) / stride + 1 : 0;
    if (L == 0) return WX_OK;
    if (!workspace || workspace_bytes < wx_conv0_channel_norm_workspace_bytes(L, C)) return WX_E_WORKSPACE;
    const bool rl = K == 10 && stride == 5;  // wav2vec2's geometry: the register-resident kernels
    const int64_t rows_per_blk = rl ? 4 * kC0R : kRows * kC0Rows;
    const int64_t nblk = (L + rows_per_blk - 1) / rows_per_blk;
    if (nblk > 65535) return WX_E_INVALID;  // (grid y; ~4.2 h of 16 kHz audio at stride 5)
    hipStream_t st = reinterpret_cast<hipStream_t>(stream);
    if (rl) {
        double* part = reinterpret_cast<double*>(workspace);
        float* ab = reinterpret_cast<float*>(part + (size_t)nblk * 2 * C);
        const dim3 grid((C + 63) / 64, (unsigned)nblk);
        hipLaunchKernelGGL((conv0_stats_rl_kernel<10, 5>), grid, dim3(256), 0, st, x, S, L, w, bias, C, part);
        hipLaunchKernelGGL(conv0_finish_kernel, dim3((C + kCols - 1) / kCols), dim3(kCols * kRows), 0, st, part,
                           (int)nblk, L, C, gamma, beta, eps, ab);
        hipLaunchKernelGGL((conv0_apply_rl_kernel<10, 5>), grid, dim3(256), 0, st, x, S, L, w, bias, C, ab, gelu, y);
        const hipError_t e = hipGetLastError();
        return e == hipSuccess ? WX_OK : (int)e;
    }
    double* part = reinterpret_cast<double*>(workspace);
    float* ab = reinterpret_cast<float*>(part + (size_t)nblk * 2 * C);
    const dim3 grid((C + kCols - 1) / kCols, (unsigned)nblk), blk(kCols * kRows);
#define WX_C0(KK)                                                                                              \
    case KK:                                                                                                   \
        hipLaunchKernelGGL(conv0_stats_kernel<KK>, grid, blk, 0, st, x, L, stride, w, bias, C, part);           \
        hipLaunchKernelGGL(conv0_finish_kernel, dim3((C + kCols - 1) / kCols), blk, 0, st, part, (int)nblk, L, C, \
                           gamma, beta, eps, ab);                                                              \
        hipLaunchKernelGGL(conv0_apply_kernel<KK>, grid, blk, 0, st, x, L, stride, w, bias, C, ab, gelu, y);    \
        break;
    switch (K) {
        WX_C0(1) WX_C0(2) WX_C0(3) WX_C0(4) WX_C0(5) WX_C0(6) WX_C0(7) WX_C0(8) WX_C0(9) WX_C0(10) WX_C0(11)
        WX_C0(12) WX_C0(13) WX_C0(14) WX_C0(15) WX_C0(16)
        default: return WX_E_INVALID;
    }
#undef WX_C0
    const hipError_t e = hipGetLastError();
    return e == hipSuccess ? WX_OK : (int)e;
}

extern "C" int wx_attention_f32(const float* q, const float* k, const float* v, float* o, int32_t B, int32_t H,
                                int32_t T, int32_t D, const int64_t* q_strides, const int64_t* k_strides,
                                const int64_t* v_strides, float scale, void* stream) {
    using namespace wxe;
    if (B < 0 || H <= 0 || T < 0 || D != 64 || !q || !k || !v || !o || !q_strides || !k_strides || !v_strides)
        return WX_E_INVALID;
    if (B == 0 || T == 0) return WX_OK;
    if ((int64_t)(T + 31) / 32 * B * H > INT32_MAX) return WX_E_INVALID;  // (one grid dimension)
    const int64_t* st[3] = {q_strides, k_strides, v_strides};
    const float* pt[3] = {q, k, v};
    for (int i = 0; i < 3; ++i) {  // 16-byte rows (float4 reads of Q / K)
        if ((reinterpret_cast<uintptr_t>(pt[i]) & 15) || (st[i][0] & 3) || (st[i][1] & 3) || (st[i][2] & 3))
            return WX_E_INVALID;
    }
    if (reinterpret_cast<uintptr_t>(o) & 15) return WX_E_INVALID;
    AttnArgs a;
    a.q = q;
    a.k = k;
    a.v = v;
    a.o = o;
    a.B = B;
    a.H = H;
    a.T = T;
    a.sqb = q_strides[0];
    a.sqh = q_strides[1];
    a.sqt = q_strides[2];
    a.skb = k_strides[0];
    a.skh = k_strides[1];
    a.skt = k_strides[2];
    a.svb = v_strides[0];
    a.svh = v_strides[1];
    a.svt = v_strides[2];
    a.scale_log2 = scale * 1.4426950408889634f;
    a.seg_rows = a.seg_units = nullptr;
    a.nseg = 0;
    const dim3 grid((unsigned)((int64_t)(T + 31) / 32 * B * H));
    hipLaunchKernelGGL((attn_f32_kernel<kAttnSplit, false>), grid, dim3(64 * kAttnSplit), 0,
                       reinterpret_cast<hipStream_t>(stream), a);
    const hipError_t e = hipGetLastError();
    return e == hipSuccess ? WX_OK : (int)e;
}


extern "C" int wx_attention_f32_packed(const float* q, const float* k, const float* v, float* o, int32_t nseg,
                                       const int32_t* seg_rows, const int32_t* seg_units, int32_t n_units,
                                       int32_t H, int32_t D, const int64_t* q_strides, const int64_t* k_strides,
                                       const int64_t* v_strides, float scale, int32_t split, void* stream) {
    using namespace wxe;
    if (nseg < 0 || H <= 0 || D != 64 || n_units < 0 || !q || !k || !v || !o || !q_strides || !k_strides ||
        !v_strides)
        return WX_E_INVALID;
    if (nseg == 0 || n_units == 0) return WX_OK;
    if (!seg_rows || !seg_units) return WX_E_INVALID;
    const int64_t* st[3] = {q_strides, k_strides, v_strides};
    const float* pt[3] = {q, k, v};
    for (int i = 0; i < 3; ++i) {  // 16-byte rows (float4 reads of Q / K)
        if ((reinterpret_cast<uintptr_t>(pt[i]) & 15) || (st[i][0] & 3) || (st[i][1] & 3)) return WX_E_INVALID;
    }
    if (reinterpret_cast<uintptr_t>(o) & 15) return WX_E_INVALID;
    AttnArgs a;
    a.q = q;
    a.k = k;
    a.v = v;
    a.o = o;
    a.B = 1;
    a.H = H;
    a.T = 0;
    a.sqb = a.skb = a.svb = 0;
    a.sqh = q_strides[0];
    a.sqt = q_strides[1];
    a.skh = k_strides[0];
    a.skt = k_strides[1];
    a.svh = v_strides[0];
    a.svt = v_strides[1];
    a.scale_log2 = scale * 1.4426950408889634f;
    a.seg_rows = seg_rows;
    a.seg_units = seg_units;
    a.nseg = nseg;
    hipStream_t s = reinterpret_cast<hipStream_t>(stream);
    // a few segments' units leave SIMDs idle unless each query tile's keys are split over waves;
    // with ~10 units per CU or more, one wave per tile (no merge) keeps them as busy
    if (split <= 0) split = n_units >= 2560 ? 1 : 4;
    switch (split) {
        case 1: hipLaunchKernelGGL((attn_f32_kernel<1, true>), dim3((unsigned)n_units), dim3(64), 0, s, a); break;
        case 2: hipLaunchKernelGGL((attn_f32_kernel<2, true>), dim3((unsigned)n_units), dim3(128), 0, s, a); break;
        case 4: hipLaunchKernelGGL((attn_f32_kernel<4, true>), dim3((unsigned)n_units), dim3(256), 0, s, a); break;
        default: return WX_E_INVALID;
    }
    const hipError_t e = hipGetLastError();
    return e == hipSuccess ? WX_OK : (int)e;
}

extern "C" int wx_add_layernorm(const float* a, const float* b, int64_t rows, int32_t D, int64_t a_stride,
                                int64_t b_stride, const float* gamma, const float* beta, float eps, float* y,
                                float* sum_out, void* stream) {
    using namespace wxe;
    if (rows < 0 || (D != 768 && D != 1024 && D != 512 && D != 256)) return WX_E_INVALID;
    if (rows == 0) return WX_OK;  // (an empty tensor may have no storage)
    if (!a || !b || !gamma || !beta || !y) return WX_E_INVALID;
    if (a_stride < D || b_stride < D || (a_stride & 3) || (b_stride & 3)) return WX_E_INVALID;
    for (const void* p : {(const void*)a, (const void*)b, (const void*)gamma, (const void*)beta, (const void*)y})
        if (reinterpret_cast<uintptr_t>(p) & 15) return WX_E_INVALID;
    if (sum_out && (reinterpret_cast<uintptr_t>(sum_out) & 15)) return WX_E_INVALID;
    hipStream_t st = reinterpret_cast<hipStream_t>(stream);
    const dim3 grid((unsigned)((rows + 3) / 4));
    switch (D) {
        case 256: hipLaunchKernelGGL(add_ln_kernel<1>, grid, dim3(256), 0, st, a, b, gamma, beta, eps, rows, a_stride, b_stride, (int64_t)D, y, sum_out); break;
        case 512: hipLaunchKernelGGL(add_ln_kernel<2>, grid, dim3(256), 0, st, a, b, gamma, beta, eps, rows, a_stride, b_stride, (int64_t)D, y, sum_out); break;
        case 768: hipLaunchKernelGGL(add_ln_kernel<3>, grid, dim3(256), 0, st, a, b, gamma, beta, eps, rows, a_stride, b_stride, (int64_t)D, y, sum_out); break;
        default: hipLaunchKernelGGL(add_ln_kernel<4>, grid, dim3(256), 0, st, a, b, gamma, beta, eps, rows, a_stride, b_stride, (int64_t)D, y, sum_out); break;
    }
    const hipError_t e = hipGetLastError();
    return e == hipSuccess ? WX_OK : (int)e;
}

extern "C" int wx_posconv_packed(const float* h, int32_t D, const float* w_packed, const float* bias, int32_t G,
                                 int32_t K, int32_t nseg, const int32_t* seg_rows, const int32_t* seg_tiles,
                                 int32_t n_tiles, int32_t residual, float* out, void* stream) {
    using namespace wxe;
    if (!h || !w_packed || !out || G <= 0 || D <= 0 || D % G || nseg < 0 || n_tiles < 0) return WX_E_INVALID;
    if (K != kPcK) return WX_E_INVALID;
    if (nseg == 0 || n_tiles == 0) return WX_OK;
    if (!seg_rows || !seg_tiles || G > 65535) return WX_E_INVALID;
    if ((reinterpret_cast<uintptr_t>(h) & 15) || (D & 3)) return WX_E_INVALID;
    PosConvArgs a;
    a.h = h;
    a.w = w_packed;
    a.bias = bias;
    a.out = out;
    a.seg_rows = seg_rows;
    a.seg_tiles = seg_tiles;
    a.nseg = nseg;
    a.D = D;
    a.residual = residual;
    hipStream_t s = reinterpret_cast<hipStream_t>(stream);
    const dim3 grid((unsigned)n_tiles, (unsigned)G);
    switch (D / G) {
        case 48: hipLaunchKernelGGL(posconv_kernel<48>, grid, dim3(256), 0, s, a); break;
        case 64: hipLaunchKernelGGL(posconv_kernel<64>, grid, dim3(256), 0, s, a); break;
        default: return WX_E_INVALID;
    }
    const hipError_t e = hipGetLastError();
    return e == hipSuccess ? WX_OK : (int)e;
}
