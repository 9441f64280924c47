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
    if (active) {
        for (int t = r; t < a.Lp; t += R) {
            const float4* src = reinterpret_cast<const float4*>(x + (int64_t)3 * t * a.C) + g;
            float4 u = src[0], v = src[G], w = src[2 * G];
            if (a.in_scale) {  // the window's input affine (a shared convolution, per-window norm)
                const float sc = a.in_scale[b];
                const float4 sh = reinterpret_cast<const float4*>(a.in_shift + (int64_t)b * a.C)[g];
                u = make_float4(u.x * sc + sh.x, u.y * sc + sh.y, u.z * sc + sh.z, u.w * sc + sh.w);
                v = make_float4(v.x * sc + sh.x, v.y * sc + sh.y, v.z * sc + sh.z, v.w * sc + sh.w);
                w = make_float4(w.x * sc + sh.x, w.y * sc + sh.y, w.z * sc + sh.z, w.w * sc + sh.w);
            }
            if (a.do_abs) {
                u = make_float4(fabsf(u.x), fabsf(u.y), fabsf(u.z), fabsf(u.w));
                v = make_float4(fabsf(v.x), fabsf(v.y), fabsf(v.z), fabsf(v.w));
                w = make_float4(fabsf(w.x), fabsf(w.y), fabsf(w.z), fabsf(w.w));
            }
            const float4 p = make_float4(nan_max(nan_max(u.x, v.x), w.x), nan_max(nan_max(u.y, v.y), w.y),
                                         nan_max(nan_max(u.z, v.z), w.z), nan_max(nan_max(u.w, v.w), w.w));
            reinterpret_cast<float4*>(y + (int64_t)t * a.C)[g] = p;
            s0 += p.x; s1 += p.y; s2 += p.z; s3 += p.w;
            q0 += (double)p.x * p.x; q1 += (double)p.y * p.y; q2 += (double)p.z * p.z; q3 += (double)p.w * p.w;
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
    for (int t = r; t < a.Lp; t += R) {
        float4* d = reinterpret_cast<float4*>(y + (int64_t)t * a.C) + g;
        const float4 p = *d;
        *d = make_float4(lrelu((p.x - mu.x) * sc.x + sh.x), lrelu((p.y - mu.y) * sc.y + sh.y),
                         lrelu((p.z - mu.z) * sc.z + sh.z), lrelu((p.w - mu.w) * sc.w + sh.w));
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
