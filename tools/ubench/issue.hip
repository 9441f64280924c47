// Issue-rate micro-benchmark (development tool): cycles per wave-instruction of candidate
// per-cell instruction mixes at a chosen occupancy.  hipcc --offload-arch=gfx950 -O3 issue.hip
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>

#define REP8(x) x x x x x x x x
// each body: 8 independent chains (v0..v15 data), repeated; counts = wave-instructions per body
#define K_ADD   REP8("v_add_f32 v0, v1, v0\n v_add_f32 v2, v3, v2\n")                          // 16
#define K_MAXV  REP8("v_max_f32 v0, v1, v0\n v_max_f32 v2, v3, v2\n")                          // 16
#define K_MAXM3 REP8("v_maximum3_f32 v0, v1, v0, v0\n v_maximum3_f32 v2, v3, v2, v2\n")        // 16
#define K_MAX3  REP8("v_max3_f32 v0, v1, v0, v0\n v_max3_f32 v2, v3, v2, v2\n")                // 16
#define K_CMPADDC REP8("v_cmp_gt_f32 vcc, v1, v0\n v_addc_co_u32 v4, vcc, v4, v4, vcc\n")      // 16
#define K_CMPCND REP8("v_cmp_gt_f32 vcc, v1, v0\n v_cndmask_b32 v4, v0, v1, vcc\n")            // 16
#define K_CMP2   REP8("v_cmp_gt_f32 vcc, v1, v0\n v_addc_co_u32 v4, vcc, v4, v4, vcc\n v_cndmask_b32 v5, v0, v1, vcc\n") // 24
#define K_CMPS   REP8("v_cmp_gt_f32_e64 s[20:21], v1, v0\n v_addc_co_u32_e64 v4, s[20:21], v4, v4, s[20:21]\n") // 16
#define K_SUBALIGN REP8("v_sub_f32 v6, v1, v0\n v_alignbit_b32 v4, v4, v6, 31\n")              // 16
#define K_PKADD REP8("v_pk_add_f32 v[0:1], v[2:3], v[0:1]\n v_pk_add_f32 v[4:5], v[6:7], v[4:5]\n") // 16
#define K_DPP   REP8("v_mov_b32_dpp v0, v1 wave_shr:1 row_mask:0xf bank_mask:0xf\n v_mov_b32_dpp v2, v3 wave_shr:1 row_mask:0xf bank_mask:0xf\n") // 16
#define K_CELL  REP8("v_add_f32 v6, v0, v10\n v_add_f32 v7, v1, v11\n v_cmp_gt_f32 vcc, v7, v6\n v_addc_co_u32 v4, vcc, v4, v4, vcc\n v_maximum3_f32 v0, v6, v7, v7\n") // 40
#define K_CELLF REP8("v_add_f32 v6, v0, v10\n v_add_f32 v7, v1, v11\n v_cmp_gt_f32 vcc, v7, v6\n v_addc_co_u32 v4, vcc, v4, v4, vcc\n v_cndmask_b32 v0, v6, v7, vcc\n") // 40
#define K_CELLM REP8("v_add_f32 v6, v0, v10\n v_add_f32 v7, v1, v11\n v_cmp_gt_f32 vcc, v7, v6\n v_addc_co_u32 v4, vcc, v4, v4, vcc\n v_max_f32 v0, v6, v7\n") // 40
#define K_CELL3 REP8("v_add_f32 v6, v0, v10\n v_add_f32 v7, v1, v11\n v_max_f32 v0, v6, v7\n") // 24
#define K_MIX  REP8("v_add_f32 v6, v0, v10\n v_maximum3_f32 v0, v6, v7, v7\n")   // 16

#define KERNEL(NAME, BODY)                                                   \
    __global__ void NAME(float* out, int iters) {                            \
        float x = threadIdx.x;                                               \
        asm volatile("v_mov_b32 v0, %0\n v_mov_b32 v1, %0\n v_mov_b32 v2, %0\n v_mov_b32 v3, %0\n v_mov_b32 v4, 0\n v_mov_b32 v5, 0\n v_mov_b32 v6, %0\n v_mov_b32 v7, %0\n v_mov_b32 v10, %0\n v_mov_b32 v11, %0" ::"v"(x) \
                     : "v0", "v1", "v2", "v3", "v4", "v5", "v6", "v7", "v10", "v11");            \
        for (int i = 0; i < iters; ++i)                                      \
            asm volatile(BODY ::: "v0", "v1", "v2", "v3", "v4", "v5", "v6", "v7", "v10", "v11", "vcc", "s20", "s21"); \
        float r;                                                             \
        asm volatile("v_add_f32 %0, v0, v4" : "=v"(r));                      \
        if (r == 12345.f) out[threadIdx.x] = r;                              \
    }

KERNEL(k_add, K_ADD)
KERNEL(k_maxv, K_MAXV)
KERNEL(k_maxm3, K_MAXM3)
KERNEL(k_max3, K_MAX3)
KERNEL(k_cmpaddc, K_CMPADDC)
KERNEL(k_cmpcnd, K_CMPCND)
KERNEL(k_cmp2, K_CMP2)
KERNEL(k_cmps, K_CMPS)
KERNEL(k_subalign, K_SUBALIGN)
KERNEL(k_pkadd, K_PKADD)
KERNEL(k_dpp, K_DPP)
KERNEL(k_cell, K_CELL)
KERNEL(k_cellf, K_CELLF)
KERNEL(k_cellm, K_CELLM)
KERNEL(k_cell3, K_CELL3)
KERNEL(k_mix, K_MIX)

int main(int argc, char** argv) {
    float* out;
    hipMalloc(&out, 4096);
    int cus = 256;
    struct { const char* n; void (*k)(float*, int); int per; } ks[] = {
        {"v_add_f32", k_add, 16}, {"v_max_f32", k_maxv, 16}, {"v_maximum3_f32", k_maxm3, 16},
        {"v_max3_f32", k_max3, 16}, {"cmp_vcc+addc", k_cmpaddc, 16}, {"cmp_vcc+cndmask", k_cmpcnd, 16},
        {"cmp+addc+cndmask", k_cmp2, 24}, {"cmp_e64+addc_e64(sgpr)", k_cmps, 16}, {"sub+alignbit", k_subalign, 16},
        {"v_pk_add_f32", k_pkadd, 16}, {"dpp mov", k_dpp, 16}, {"cell(add,add,cmp,addc,maximum3)", k_cell, 40},
        {"cell(add,add,cmp,addc,cndmask)", k_cellf, 40}, {"cell(add,add,cmp,addc,max)", k_cellm, 40},
        {"cell3(add,add,max)", k_cell3, 24}, {"add+maximum3", k_mix, 16}};
    const int iters = 2000;
    for (int wps : {1, 2, 4, 8}) {
        printf("== waves/SIMD %d\n", wps);
        for (auto& k : ks) {
            hipLaunchKernelGGL(k.k, dim3(cus * 4 * wps), dim3(64), 0, 0, out, 10);
            hipEvent_t a, b;
            hipEventCreate(&a);
            hipEventCreate(&b);
            hipEventRecord(a);
            hipLaunchKernelGGL(k.k, dim3(cus * 4 * wps), dim3(64), 0, 0, out, iters);
            hipEventRecord(b);
            hipEventSynchronize(b);
            float ms;
            hipEventElapsedTime(&ms, a, b);
            // cycles at 2.4 GHz per wave-instruction per SIMD
            double inst_per_simd = (double)wps * iters * k.per;
            printf("  %-34s %6.2f cyc/inst/SIMD  (%.3f ms)\n", k.n, ms * 1e-3 * 2.4e9 / inst_per_simd, ms);
        }
    }
    return 0;
}
