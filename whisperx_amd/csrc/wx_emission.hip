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
