// wx_vad.hip — gfx950 kernels of the VAD producer (reference
// whisperx/vad.py:198-240, the pyannote segmentation model's forward): the epilogue of each of
// SincNet's three stages, fused.
//
// pyannote's SincNet stage is conv -> (|.| after the sinc filterbank) -> MaxPool1d(3, 3) ->
// InstanceNorm1d(affine) -> LeakyReLU.  The GEMM route (vad_model.conv1d_batched) leaves the
// conv output time-major, [B windows, L, C]; torch then ran four memory-bound passes over it —
// abs, max-pool, instance norm (two kernels), leaky ReLU — each reading and writing the whole
// first-stage activation (5.2 GB per 2,048-window batch): ~36% of the producer's GPU time
// (profiles/r3_vad1h_kernel_stats.csv).  Here one workgroup per window:
//   phase 1: pooled[t, c] = max over rows 3t .. 3t+2 of (|)x(|) -> written time-major, with
//            per-channel fp64 sums and sums of squares;
//   phase 2: mean / biased variance per channel (InstanceNorm1d, eps), then
//            y = leaky_relu((pooled - mean) * (rstd * gamma) + beta) in place (the centring
//            first, as InstanceNorm1d: folding the mean into the shift loses the digits of a
//            near-constant channel).
// HBM: one read of x, one write + one read + one write of the pooled third.
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdint.h>

#include "../../include/wx_align.h"

namespace wxv {

constexpr int kThreads = 256;
constexpr int kMaxC = 128;  // channels per window (float4 groups: kMaxC / 4)

struct SincArgs {
    const float* x;    // [B][L][C] (window stride xb elements, row stride C)
    int64_t xb;
    int L, C, Lp;      // Lp = L / 3 pooled rows
    int do_abs;
    const float* gamma;
    const float* beta;
    float eps, slope;
    float* y;          // [B][Lp][C] contiguous
    const float* in_scale;  // [B] or null: x * in_scale[b] + in_shift[b][c] before |.|
    const float* in_shift;  // [B][C] or null
};

__device__ __forceinline__ float nan_max(float a, float b) { return __builtin_elementwise_maximum(a, b); }

__global__ __launch_bounds__(kThreads) void sinc_stage_kernel(SincArgs a) {
    const int b = blockIdx.x;
    const int G = a.C >> 2;              // float4 groups per row
    const int R = kThreads / G;          // pooled rows per pass
    const int tid = (int)threadIdx.x;
    const int g = tid % G, r = tid / G;
    const bool active = r < R;
    const float* x = a.x + (int64_t)b * a.xb;
    float* y = a.y + (int64_t)b * a.Lp * a.C;
    double s0 = 0.0, s1 = 0.0, s2 = 0.0, s3 = 0.0, q0 = 0.0, q1 = 0.0, q2 = 0.0, q3 = 0.0;
    // (the window's input affine: a shared convolution with a per-window norm)
    const float sc_in = a.in_scale ? a.in_scale[b] : 1.0f;
    const float4 sh_in = a.in_scale ? reinterpret_cast<const float4*>(a.in_shift + (int64_t)b * a.C)[g]
                                    : make_float4(0.f, 0.f, 0.f, 0.f);
    auto pool = [&](float4 u, float4 v, float4 w) {
        if (a.in_scale) {
            u = make_float4(u.x * sc_in + sh_in.x, u.y * sc_in + sh_in.y, u.z * sc_in + sh_in.z, u.w * sc_in + sh_in.w);
            v = make_float4(v.x * sc_in + sh_in.x, v.y * sc_in + sh_in.y, v.z * sc_in + sh_in.z, v.w * sc_in + sh_in.w);
            w = make_float4(w.x * sc_in + sh_in.x, w.y * sc_in + sh_in.y, w.z * sc_in + sh_in.z, w.w * sc_in + sh_in.w);
        }
        if (a.do_abs) {
            u = make_float4(fabsf(u.x), fabsf(u.y), fabsf(u.z), fabsf(u.w));
            v = make_float4(fabsf(v.x), fabsf(v.y), fabsf(v.z), fabsf(v.w));
            w = make_float4(fabsf(w.x), fabsf(w.y), fabsf(w.z), fabsf(w.w));
        }
        return make_float4(nan_max(nan_max(u.x, v.x), w.x), nan_max(nan_max(u.y, v.y), w.y),
                           nan_max(nan_max(u.z, v.z), w.z), nan_max(nan_max(u.w, v.w), w.w));
    };
    auto acc = [&](float4 p) {  // (rows of a thread in increasing order)
        s0 += p.x; s1 += p.y; s2 += p.z; s3 += p.w;
        q0 += (double)p.x * p.x; q1 += (double)p.y * p.y; q2 += (double)p.z * p.z; q3 += (double)p.w * p.w;
    };
    // four pooled rows per thread and pass: twelve 16-byte loads in flight instead of three (a
    // latency-bound 3.7 TB/s before)
    constexpr int kU = 4;
    int t = r;
    if (active) {
        for (; t + (kU - 1) * R < a.Lp; t += kU * R) {
            float4 u[kU], v[kU], w[kU];
#pragma unroll
            for (int k = 0; k < kU; ++k) {
                const float4* src = reinterpret_cast<const float4*>(x + (int64_t)3 * (t + k * R) * a.C) + g;
                u[k] = src[0];
                v[k] = src[G];
                w[k] = src[2 * G];
            }
#pragma unroll
            for (int k = 0; k < kU; ++k) {
                const float4 p = pool(u[k], v[k], w[k]);
                reinterpret_cast<float4*>(y + (int64_t)(t + k * R) * a.C)[g] = p;
                acc(p);
            }
        }
        for (; t < a.Lp; t += R) {
            const float4* src = reinterpret_cast<const float4*>(x + (int64_t)3 * t * a.C) + g;
            const float4 p = pool(src[0], src[G], src[2 * G]);
            reinterpret_cast<float4*>(y + (int64_t)t * a.C)[g] = p;
            acc(p);
        }
    }
    __shared__ double red[kThreads / 4][8];  // (R <= kThreads / 4 when G >= 4)
    __shared__ float coef[3][kMaxC];  // rstd * gamma, mean, beta
    // channel sums: row r's partials per group, then one thread per channel adds them in row order
    __shared__ double part[2][kMaxC];
    for (int rr = 0; rr < R; ++rr) {
        if (active && r == rr) {
            red[g][0] = s0; red[g][1] = s1; red[g][2] = s2; red[g][3] = s3;
            red[g][4] = q0; red[g][5] = q1; red[g][6] = q2; red[g][7] = q3;
        }
        __syncthreads();
        if (tid < a.C) {
            const int gg = tid >> 2, k = tid & 3;
            const double ps = red[gg][k], pq = red[gg][4 + k];
            part[0][tid] = rr == 0 ? ps : part[0][tid] + ps;
            part[1][tid] = rr == 0 ? pq : part[1][tid] + pq;
        }
        __syncthreads();
    }
    if (tid < a.C) {
        const double n = (double)a.Lp;
        const double mean = part[0][tid] / n;
        const double var = fmax(part[1][tid] / n - mean * mean, 0.0);  // biased, as InstanceNorm1d
        const double rstd = 1.0 / sqrt(var + (double)a.eps);
        const double gm = a.gamma ? (double)a.gamma[tid] : 1.0, bt = a.beta ? (double)a.beta[tid] : 0.0;
        coef[0][tid] = (float)(rstd * gm);
        coef[1][tid] = (float)mean;
        coef[2][tid] = (float)bt;
    }
    // this thread's pooled writes are re-read by this thread only; the barrier orders coef
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
    __syncthreads();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
    if (!active) return;
    const float4 sc = make_float4(coef[0][4 * g], coef[0][4 * g + 1], coef[0][4 * g + 2], coef[0][4 * g + 3]);
    const float4 mu = make_float4(coef[1][4 * g], coef[1][4 * g + 1], coef[1][4 * g + 2], coef[1][4 * g + 3]);
    const float4 sh = make_float4(coef[2][4 * g], coef[2][4 * g + 1], coef[2][4 * g + 2], coef[2][4 * g + 3]);
    const float sl = a.slope;
    auto lrelu = [sl](float v) { return v > 0.0f ? v : v * sl; };
    auto norm = [&](float4 p) {
        return make_float4(lrelu((p.x - mu.x) * sc.x + sh.x), lrelu((p.y - mu.y) * sc.y + sh.y),
                           lrelu((p.z - mu.z) * sc.z + sh.z), lrelu((p.w - mu.w) * sc.w + sh.w));
    };
    t = r;
    for (; t + (kU - 1) * R < a.Lp; t += kU * R) {
        float4 p[kU];
#pragma unroll
        for (int k = 0; k < kU; ++k) p[k] = reinterpret_cast<const float4*>(y + (int64_t)(t + k * R) * a.C)[g];
#pragma unroll
        for (int k = 0; k < kU; ++k) reinterpret_cast<float4*>(y + (int64_t)(t + k * R) * a.C)[g] = norm(p[k]);
    }
    for (; t < a.Lp; t += R) {
        float4* d = reinterpret_cast<float4*>(y + (int64_t)t * a.C) + g;
        *d = norm(*d);
    }
}

// ------------------------------------------------------------------------------------
// SincNet's k = 5 convolutions (pyannote SincNet stages 2 and 3: Conv1d(80, 60, 5) and
// Conv1d(60, 60, 5), no padding), time-major, every window of a batch in one launch.  As tap
// GEMMs (vad_model.conv1d_batched) each was 5 passes over the [B L, Cin] activation with the
// [B L, 60] output read and written per tap (memory-bound, ~33 ms per hour of audio).  Here
// one block per (window, 128 output frames): the 132 input rows sit in LDS once, the taps'
// [Cin, 64] weight slabs stream through one LDS slab, 4 waves x 32 frames x 64
// outputs (60 used) on v_mfma_f32_16x16x4_f32; + bias, written once.  fp32 (fma chains: not
// bit-identical to the GEMM route, tests compare at fp32 tolerance).
constexpr int kCkFrames = 128;

// One weight slab in LDS (round 6): a block is 64 KB (Cin 80), so two blocks share a CU and
// one's slab load and barriers hide under the other's MFMAs.  (Round 5 double-buffered the slab
// — 84 KB, one block per CU, the next tap's store overlapped inside the block: 1 ms per hour
// slower.)

template <int CINP, int KT>
__global__ __launch_bounds__(256) void conv_taps_kernel(const float* __restrict__ x, int Cin, int L,
                                                        const float* __restrict__ wp /* [KT][CINP/4][64][4] */,
                                                        const float* __restrict__ bias, float* __restrict__ y,
                                                        int Cout, int Lout) {
    typedef float f32x4 __attribute__((ext_vector_type(4)));
    constexpr int RS = CINP + 4;
    constexpr int WR = kCkFrames + KT - 1;
    constexpr int NOB = 4, NIC = CINP / 16;
    constexpr int NB4 = CINP * 64 / 4;
    constexpr int PER = (NB4 + 255) / 256;
    __shared__ __attribute__((aligned(16))) float xa[WR * RS];
    __shared__ __attribute__((aligned(16))) float wb[CINP * 64];
    const int b = blockIdx.y;
    const int t0 = blockIdx.x * kCkFrames;
    const float* xb = x + (int64_t)b * L * Cin;
    const int c4n = Cin / 4;
    for (int e = threadIdx.x; e < WR * (CINP / 4); e += 256) {
        const int r = e / (CINP / 4), c4 = e - r * (CINP / 4);
        const int t = t0 + r;
        float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
        if (t < L && c4 < c4n) v = *reinterpret_cast<const float4*>(xb + (int64_t)t * Cin + 4 * c4);
        *reinterpret_cast<float4*>(xa + r * RS + 4 * c4) = v;
    }
    const float4* wg = reinterpret_cast<const float4*>(wp);
    // the next tap's slab in five named registers (a float4 array here stayed a stack object in
    // scratch memory: each tap stored it there and loaded it back after the barrier)
    static_assert(NB4 % 256 == 0 && PER <= 5, "conv_taps: whole float4 rows per thread");
    float4 b0, b1, b2, b3, b4;
    auto bload = [&](int j) {
        const float4* src = wg + (int64_t)j * NB4 + threadIdx.x;
        b0 = src[0];
        b1 = src[256];
        b2 = src[512];
        b3 = src[768];
        if constexpr (PER > 4) b4 = src[1024];
    };
    auto bstore = [&]() {
        float4* dst = reinterpret_cast<float4*>(wb) + threadIdx.x;
        dst[0] = b0;
        dst[256] = b1;
        dst[512] = b2;
        dst[768] = b3;
        if constexpr (PER > 4) dst[1024] = b4;
    };
    bload(0);
    bstore();
    __syncthreads();
    const int l = threadIdx.x & 63, wv = threadIdx.x >> 6, q = l >> 4, r16 = l & 15;
    f32x4 acc[2][NOB];
#pragma unroll
    for (int fb = 0; fb < 2; ++fb)
#pragma unroll
        for (int ob = 0; ob < NOB; ++ob) acc[fb][ob] = f32x4{0.f, 0.f, 0.f, 0.f};
    const float* xrow = xa + (wv * 32 + r16) * RS + 4 * q;
#pragma unroll
    for (int j = 0; j < KT; ++j) {
        if (j + 1 < KT) bload(j + 1);
        // (issued here, under the tap's MFMAs: hipcc otherwise sinks the loads to the store
        // after the barrier, a global round trip per tap)
        __builtin_amdgcn_sched_barrier(0);
        const float* bb = wb + (q * 64 + r16) * 4;
#pragma unroll
        for (int ic = 0; ic < NIC; ++ic) {
            float4 av[2], bv[NOB];
#pragma unroll
            for (int fb = 0; fb < 2; ++fb) av[fb] = *reinterpret_cast<const float4*>(xrow + (16 * fb + j) * RS + 16 * ic);
#pragma unroll
            for (int ob = 0; ob < NOB; ++ob) bv[ob] = *reinterpret_cast<const float4*>(bb + (ic * 4 * 64 + 16 * ob) * 4);
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
        __syncthreads();  // every wave is done with tap j's slab
        if (j + 1 < KT) {
            bstore();
            __syncthreads();
        }
    }
    float* yb = y + (int64_t)b * Lout * Cout;
#pragma unroll
    for (int fb = 0; fb < 2; ++fb)
#pragma unroll
        for (int v = 0; v < 4; ++v) {
            const int t = t0 + wv * 32 + 16 * fb + 4 * q + v;
            if (t >= Lout) continue;
#pragma unroll
            for (int ob = 0; ob < NOB; ++ob) {
                const int c = 16 * ob + r16;
                if (c < Cout) yb[(int64_t)t * Cout + c] = acc[fb][ob][v] + (bias ? bias[c] : 0.f);
            }
        }
}

// ------------------------------------------------------------------------------------
// SincNet's filterbank over a waveform span (the shared-sinc route: pyannote SincNet stage 1,
// a bias-free Conv1d(1, C, k = 251, stride 10), run once per batch of overlapping windows):
// y[t][c] = sum_{j < KP} x[S t + j] w[j][c], KP = k zero-padded to a multiple of 4 (zeros past
// the end of x), t < (n - k) / S + 1.  As a
// GEMM on the unfold view (rows overlap: stride S < KP) torch first copied every patch row
// out (~1 GB chunks, 1.7 ms per hour of audio) and then multiplied (3.0 ms).  Here the rows
// are read where they lie: a block stages the 256 S + KP samples of its 256 output rows in
// LDS once; wave w owns channels 16 w .. 16 w + 15 and keeps their KP x 16 filter taps as
// v_mfma_f32_16x16x4_f32 B fragments in registers for the whole block; each MFMA's A fragment
// (16 rows x 4 taps) is one LDS read per lane at S (row) + tap.  fp32 (tolerance-equal to
// the GEMM: a different summation order).
constexpr int kSfRows = 256;   // output rows per block
constexpr int kSfMaxS = 16;    // stride bound of the LDS window

template <int NT, int KP>  // NT 16-channel tiles (C = 16 NT), KP padded taps
__global__ __launch_bounds__(64 * NT) void sinc_fb_kernel(const float* __restrict__ x, int64_t n, int S,
                                                          const float* __restrict__ w /* [KP][16 NT] */,
                                                          float* __restrict__ y, int64_t F) {
    typedef float f32x4 __attribute__((ext_vector_type(4)));
    constexpr int C = 16 * NT, NS = KP / 4;
    static_assert(KP % 4 == 0, "taps padded to a multiple of 4");
    __shared__ float xs[kSfRows * kSfMaxS + KP];
    const int64_t t0 = (int64_t)blockIdx.x * kSfRows;
    const int64_t s0 = t0 * S;
    const int nw = kSfRows * S + KP;
    for (int i = (int)threadIdx.x; i < nw; i += 64 * NT) xs[i] = s0 + i < n ? x[s0 + i] : 0.f;
    const int l = (int)threadIdx.x & 63, wv = (int)threadIdx.x >> 6, r16 = l & 15, kq = l >> 4;
    float b[NS];  // B[k = kq][col = r16] of tap group s: w[4 s + kq][16 wv + r16]
#pragma unroll
    for (int s = 0; s < NS; ++s) b[s] = w[(4 * s + kq) * C + 16 * wv + r16];
    __syncthreads();
    // two row tiles at a time (two independent accumulator chains)
    for (int rt = 0; rt < kSfRows / 16; rt += 2) {
        f32x4 a0 = {0.f, 0.f, 0.f, 0.f}, a1 = {0.f, 0.f, 0.f, 0.f};
        const float* x0 = xs + S * (16 * rt + r16) + kq;
        const float* x1 = x0 + 16 * S;
#pragma unroll
        for (int s = 0; s < NS; ++s) {
            a0 = __builtin_amdgcn_mfma_f32_16x16x4f32(x0[4 * s], b[s], a0, 0, 0, 0);
            a1 = __builtin_amdgcn_mfma_f32_16x16x4f32(x1[4 * s], b[s], a1, 0, 0, 0);
        }
        // D[row 4 kq + v][col r16]
#pragma unroll
        for (int v = 0; v < 4; ++v) {
            const int64_t t = t0 + 16 * rt + 4 * kq + v;
            if (t < F) y[t * C + 16 * wv + r16] = a0[v];
            if (t + 16 < F) y[(t + 16) * C + 16 * wv + r16] = a1[v];
        }
    }
}

// ------------------------------------------------------------------------------------
// PyanNet's bidirectional LSTM layer (pyannote segmentation, called by vad.py:198-240), one
// persistent kernel per layer for both directions.  MIOpen ran it as 293 time steps x 2
// directions of a [B, 128] x [128, 512] GEMM launch plus a gate-update launch (~37 k launches
// per hour of audio, ~29% of the producer's GPU time).  Here the input projection of every
// step (x W_ih^T + b_ih + b_hh, both directions) is one GEMM before the call (xp), and one
// workgroup carries 16 sequences of one direction through all T steps: per step
//   gates[16, 512] = xp[t] + h_{t-1} W_hh^T     (v_mfma_f32_16x16x4_f32, W_hh's fragments held
//                                               in registers for the whole sequence)
//   i, f, o = sigmoid, g = tanh;  c = f c + i g;  h = o tanh(c) -> LDS (next step's A operand)
//   and y[b, t, d H + u].
// Round 6: wave w owns hidden units 32 w .. 32 w + 31 across all four gates (tiles 2 g + half:
// gate g's columns 128 g + 32 w + 16 half + 0..15), so a lane holds i, f, g, o of the same
// (sequence, unit) in its own accumulators and the cell update is lane-local: one barrier per
// step (h into a ping-pong LDS buffer) instead of the gate activations' LDS round trip and two
// barriers (round 5: wave w computed gate w for all units).  Same MFMA order per gate value and
// the same activation functions as before: bit-identical outputs.
// fp32 throughout (fma chains in the MFMA, not bit-identical to MIOpen's; tests compare with
// torch.nn.LSTM at fp32 tolerance).  H = 128 (PyanNet).
constexpr int kLH = 128;  // hidden size
constexpr int kLR = 16;   // sequences per workgroup

// Gate activations with the hardware reciprocal (v_rcp_f32, ~1 ulp) instead of the IEEE
// division sequence (v_div_scale / v_rcp / v_div_fmas / v_div_fixup: ~10 instructions) and
// of OCML's branchy tanhf: the gate phase ran 24 divisions and 16 tanh per lane and step
// beside the step's 256 MFMAs.  tanh(x) = 2 sigmoid(2x) - 1 (absolute error ~1e-7 near 0;
// +-1 and NaN at the extremes as tanhf).  Tolerance-equal to torch.nn.LSTM (tests).
__device__ __forceinline__ float sigmoid_f(float x) { return __builtin_amdgcn_rcpf(1.0f + __expf(-x)); }
__device__ __forceinline__ float tanh_f(float x) { return 2.0f * __builtin_amdgcn_rcpf(1.0f + __expf(-2.0f * x)) - 1.0f; }

__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(1, 1))) void lstm_layer_kernel(
    const float* __restrict__ xp /* [B][T][2][4H] */, const float* __restrict__ whh /* [2][4H][H] */,
    float* __restrict__ y /* [B][T][2H] */, int B, int T) {
    typedef float f32x4 __attribute__((ext_vector_type(4)));
    constexpr int RS = kLH + 4;  // h row stride in LDS (floats)
    __shared__ __attribute__((aligned(16))) float hs[2][kLR * RS];  // ping-pong by step parity
    const int d = blockIdx.y;
    const int b0 = blockIdx.x * kLR;
    const int l = threadIdx.x & 63, w = threadIdx.x >> 6, q = l >> 4, r16 = l & 15;
    // gate column of tile tt = 2 g + half: 128 g + 32 w + 16 half + r16
    auto col = [&](int tt) { return 128 * (tt >> 1) + 32 * w + 16 * (tt & 1) + r16; };
    // this wave's W_hh fragments, kept for the whole sequence: rows col(tile), k = 16 kk + 4 q .. + 3
    const float* wd = whh + (int64_t)d * 4 * kLH * kLH;
    float4 wf[8][8];  // [tile][kk]
#pragma unroll
    for (int tile = 0; tile < 8; ++tile)
#pragma unroll
        for (int kk = 0; kk < 8; ++kk)
            wf[tile][kk] = *reinterpret_cast<const float4*>(wd + (int64_t)col(tile) * kLH + 16 * kk + 4 * q);
    for (int i = threadIdx.x; i < kLR * RS; i += 256) hs[0][i] = 0.f;
    // cell state of (sequence 4 q + v, unit 32 w + 16 half + r16): c[half][v]
    float c[2][4];
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int v = 0; v < 4; ++v) c[i][v] = 0.f;
    __syncthreads();
    // xp of a step: accumulator (tile, v) <-> sequence 4 q + v, column col(tile); the next step's
    // are loaded while this step's MFMAs run
    float xn[8][4];
    auto load_xp = [&](int s) {
        const int t = d ? T - 1 - s : s;
#pragma unroll
        for (int v = 0; v < 4; ++v) {
            const int b = min(b0 + 4 * q + v, B - 1);
            const float* xr = xp + (((int64_t)b * T + t) * 2 + d) * 4 * kLH;
#pragma unroll
            for (int tile = 0; tile < 8; ++tile) xn[tile][v] = xr[col(tile)];
        }
    };
    load_xp(0);
    for (int s = 0; s < T; ++s) {
        const int t = d ? T - 1 - s : s;
        const float* hr = hs[s & 1];
        float* hw = hs[(s + 1) & 1];
        f32x4 acc[8];
#pragma unroll
        for (int tile = 0; tile < 8; ++tile)
#pragma unroll
            for (int v = 0; v < 4; ++v) acc[tile][v] = xn[tile][v];
        if (s + 1 < T) load_xp(s + 1);
#pragma unroll
        for (int kk = 0; kk < 8; ++kk) {
            const float4 a = *reinterpret_cast<const float4*>(hr + r16 * RS + 16 * kk + 4 * q);
#pragma unroll
            for (int tile = 0; tile < 8; ++tile) {
                acc[tile] = __builtin_amdgcn_mfma_f32_16x16x4f32(a.x, wf[tile][kk].x, acc[tile], 0, 0, 0);
                acc[tile] = __builtin_amdgcn_mfma_f32_16x16x4f32(a.y, wf[tile][kk].y, acc[tile], 0, 0, 0);
                acc[tile] = __builtin_amdgcn_mfma_f32_16x16x4f32(a.z, wf[tile][kk].z, acc[tile], 0, 0, 0);
                acc[tile] = __builtin_amdgcn_mfma_f32_16x16x4f32(a.w, wf[tile][kk].w, acc[tile], 0, 0, 0);
            }
        }
        // gates (PyTorch order i, f, g, o) and the cell update, lane-local
#pragma unroll
        for (int half = 0; half < 2; ++half) {
            const int u = 32 * w + 16 * half + r16;
#pragma unroll
            for (int v = 0; v < 4; ++v) {
                const float ig = sigmoid_f(acc[half][v]), fg = sigmoid_f(acc[2 + half][v]);
                const float gg = tanh_f(acc[4 + half][v]), og = sigmoid_f(acc[6 + half][v]);
                c[half][v] = fg * c[half][v] + ig * gg;
                const float h = og * tanh_f(c[half][v]);
                hw[(4 * q + v) * RS + u] = h;
                const int b = b0 + 4 * q + v;
                if (b < B) y[((int64_t)b * T + t) * 2 * kLH + d * kLH + u] = h;
            }
        }
        __syncthreads();  // h_t complete in hw before any wave reads it as the next A operand
    }
}

}  // namespace wxv

extern "C" int wx_sincnet_stage_ex(const float* x, int64_t B, int64_t L, int32_t C, int64_t x_window_stride,
                                   int32_t do_abs, const float* in_scale, const float* in_shift, const float* gamma,
                                   const float* beta, float eps, float slope, float* y, void* stream) {
    using namespace wxv;
    // (windows may overlap: x_window_stride < L * C reads a shared time-major output)
    if (B < 0 || L < 0 || C <= 0 || C > kMaxC || (C & 3) || x_window_stride < 0) return WX_E_INVALID;
    if (L / 3 > 0x7fffffff || B > 0x7fffffff || (!in_scale != !in_shift)) return WX_E_INVALID;
    const int Lp = (int)(L / 3);
    if (B == 0 || Lp == 0) return WX_OK;  // (an empty output may have no storage)
    if (!x || !y || (reinterpret_cast<uintptr_t>(x) & 15) || (reinterpret_cast<uintptr_t>(y) & 15) ||
        (x_window_stride & 3) || (in_shift && (reinterpret_cast<uintptr_t>(in_shift) & 15)))
        return WX_E_INVALID;
    SincArgs a;
    a.x = x;
    a.xb = x_window_stride;
    a.L = (int)L;
    a.C = C;
    a.Lp = Lp;
    a.do_abs = do_abs ? 1 : 0;
    a.gamma = gamma;
    a.beta = beta;
    a.eps = eps;
    a.slope = slope;
    a.y = y;
    a.in_scale = in_scale;
    a.in_shift = in_shift;
    hipLaunchKernelGGL(sinc_stage_kernel, dim3((unsigned)B), dim3(kThreads), 0, reinterpret_cast<hipStream_t>(stream), a);
    const hipError_t e = hipGetLastError();
    return e == hipSuccess ? WX_OK : (int)e;
}

extern "C" int wx_sincnet_stage(const float* x, int64_t B, int64_t L, int32_t C, int64_t x_window_stride,
                                int32_t do_abs, const float* gamma, const float* beta, float eps, float slope,
                                float* y, void* stream) {
    if (x_window_stride < L * (int64_t)C) return WX_E_INVALID;
    return wx_sincnet_stage_ex(x, B, L, C, x_window_stride, do_abs, nullptr, nullptr, gamma, beta, eps, slope, y,
                               stream);
}

extern "C" int wx_lstm_bidir_layer(const float* xp, const float* whh, float* y, int64_t B, int64_t T, int32_t H,
                                   void* stream) {
    using namespace wxv;
    if (B < 0 || T < 0 || H != kLH || !xp || !whh || !y) return WX_E_INVALID;
    if (B == 0 || T == 0) return WX_OK;
    if ((reinterpret_cast<uintptr_t>(whh) & 15) || (reinterpret_cast<uintptr_t>(y) & 15)) return WX_E_INVALID;
    if ((B + kLR - 1) / kLR > 65535 * 1024L) return WX_E_INVALID;
    const dim3 grid((unsigned)((B + kLR - 1) / kLR), 2);
    hipLaunchKernelGGL(lstm_layer_kernel, grid, dim3(256), 0, reinterpret_cast<hipStream_t>(stream), xp, whh, y,
                       (int)B, (int)T);
    const hipError_t e = hipGetLastError();
    return e == hipSuccess ? WX_OK : (int)e;
}

extern "C" int wx_sinc_filterbank(const float* x, int64_t n, int32_t stride, const float* w_padded, int32_t C,
                                  int32_t K, int32_t KP, float* y, void* stream) {
    using namespace wxv;
    if (n < 0 || stride <= 0 || stride > kSfMaxS || K <= 0 || K > KP || !x || !w_padded || !y) return WX_E_INVALID;
    if (n < K) return WX_OK;  // no output row
    const int64_t F = (n - K) / stride + 1;
    if ((F + kSfRows - 1) / kSfRows > 0x7fffffff) return WX_E_INVALID;
    hipStream_t s = reinterpret_cast<hipStream_t>(stream);
    const dim3 grid((unsigned)((F + kSfRows - 1) / kSfRows));
    if (C == 80 && KP == 260)
        hipLaunchKernelGGL((sinc_fb_kernel<5, 260>), grid, dim3(64 * 5), 0, s, x, n, (int)stride, w_padded, y, F);
    else
        return WX_E_INVALID;
    const hipError_t e = hipGetLastError();
    return e == hipSuccess ? WX_OK : (int)e;
}

extern "C" int wx_conv1d_taps_tm(const float* x, int64_t B, int64_t L, int32_t Cin, const float* w_packed,
                                 const float* bias, int32_t Cout, int32_t K, float* y, void* stream) {
    using namespace wxv;
    if (B < 0 || L < 0 || Cin <= 0 || (Cin & 3) || Cout <= 0 || Cout > 64 || !x || !w_packed || !y) return WX_E_INVALID;
    const int64_t Lout = L >= K ? L - K + 1 : 0;
    if (B == 0 || Lout == 0) return WX_OK;
    if ((reinterpret_cast<uintptr_t>(x) & 15) || B > 65535 || L > INT32_MAX) return WX_E_INVALID;
    hipStream_t s = reinterpret_cast<hipStream_t>(stream);
    const dim3 grid((unsigned)((Lout + kCkFrames - 1) / kCkFrames), (unsigned)B);
    if (K == 5 && Cin <= 64)
        hipLaunchKernelGGL((conv_taps_kernel<64, 5>), grid, dim3(256), 0, s, x, Cin, (int)L, w_packed, bias, y, Cout,
                           (int)Lout);
    else if (K == 5 && Cin <= 80)
        hipLaunchKernelGGL((conv_taps_kernel<80, 5>), grid, dim3(256), 0, s, x, Cin, (int)L, w_packed, bias, y, Cout,
                           (int)Lout);
    else
        return WX_E_INVALID;
    const hipError_t e = hipGetLastError();
    return e == hipSuccess ? WX_OK : (int)e;
}
