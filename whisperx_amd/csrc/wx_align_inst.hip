// wx_align_inst.hip — explicit instantiations of the fused-DP, split and get_trellis kernel
// templates (wx_align_dp.h), one launcher per (bucket, row width).  Compiled once per shard
// (-DWX_SHARD=0..7) so that the ~90 kernel instantiations build in parallel; without
// WX_SHARD every instantiation is compiled (a single-TU build, e.g. WX_PHASE_TIMING).
#include "wx_align_dp.h"

namespace wx {

template <int C, int VS, int W, int H>
void launch_align_dp(dim3 grid, hipStream_t s, const AlignArgs& a) {
    hipLaunchKernelGGL((align_dp_kernel<C, VS, W, H>), grid, dim3(kWave * (W + H)), 0, s, a);
}
template <int C, int VS, int W>
void launch_align_split(dim3 grid, hipStream_t s, const AlignArgs& a) {
    hipLaunchKernelGGL((align_dp_split_kernel<C, VS, W>), grid, dim3(kWave * kSplitWaves), 0, s, a);
}
template <int C, int VS, int W>
void launch_trellis(dim3 grid, hipStream_t s, const TrellisArgs& a) {
    hipLaunchKernelGGL((trellis_kernel<C, VS, W>), grid, dim3(kWave * W), 0, s, a);
}

#ifdef WX_DEV_V32
#define WX_EACH_VS(M, ...) M(32, __VA_ARGS__)
#else
#define WX_EACH_VS(M, ...) M(32, __VA_ARGS__) M(64, __VA_ARGS__) M(kGatherVS, __VA_ARGS__)
#endif
#define WX_I_ALIGN(VS, C, W, H) template void launch_align_dp<C, VS, W, H>(dim3, hipStream_t, const AlignArgs&);
#define WX_I_SPLIT(VS, C, W) template void launch_align_split<C, VS, W>(dim3, hipStream_t, const AlignArgs&);
#define WX_I_TR(VS, C, W) template void launch_trellis<C, VS, W>(dim3, hipStream_t, const TrellisArgs&);
#define WX_ALIGN(C, W, H) WX_EACH_VS(WX_I_ALIGN, C, W, H)
#define WX_SPLIT(C, W) WX_EACH_VS(WX_I_SPLIT, C, W)
#define WX_TR(C, W) WX_EACH_VS(WX_I_TR, C, W)

// Every bucket of WX_BUCKETS / WX_SPLIT_BUCKETS (wx_align_dp.h) must appear once below; a
// missing one fails at link time (undefined launcher).
#if !defined(WX_SHARD) || WX_SHARD == 0
WX_ALIGN(1, 1, 0) WX_ALIGN(2, 1, 0) WX_ALIGN(4, 1, 0)
WX_TR(1, 1) WX_TR(2, 1) WX_TR(4, 1)
#endif
#if !defined(WX_SHARD) || WX_SHARD == 1
WX_ALIGN(6, 1, 0) WX_ALIGN(8, 1, 0)
WX_TR(6, 1) WX_TR(8, 1)
#endif
#if !defined(WX_SHARD) || WX_SHARD == 2
WX_ALIGN(8, 2, 0) WX_ALIGN(8, 4, 0)
WX_TR(8, 2) WX_TR(8, 4)
#endif
#if !defined(WX_SHARD) || WX_SHARD == 3
WX_ALIGN(8, 8, 0) WX_ALIGN(16, 8, 0)
WX_TR(8, 8) WX_TR(16, 8)
#endif
#if !defined(WX_SHARD) || WX_SHARD == 4
WX_ALIGN(32, 8, 0)
WX_TR(32, 8)
#endif
#if !defined(WX_SHARD) || WX_SHARD == 5
WX_ALIGN(1, 3, 1) WX_ALIGN(1, 7, 1) WX_ALIGN(2, 7, 1)
#endif
#if !defined(WX_SHARD) || WX_SHARD == 6
WX_ALIGN(4, 7, 1) WX_ALIGN(8, 7, 1)
#endif
#if !defined(WX_SHARD) || WX_SHARD == 7
WX_SPLIT(1, 3) WX_SPLIT(1, 4) WX_SPLIT(2, 3) WX_SPLIT(4, 3)
#endif

}  // namespace wx
