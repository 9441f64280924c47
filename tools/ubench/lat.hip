// Dependent-latency micro-benchmark (development tool): cycles (s_memtime) per instruction
// of a single wave running K interleaved dependent chains.  hipcc --offload-arch=gfx950 -O3
#include <hip/hip_runtime.h>
#include <stdio.h>

#define R4(x) x x x x
#define R16(x) R4(x) R4(x) R4(x) R4(x)
#define KER(NAME, BODY, PER)                                                                   \
    __global__ void NAME(unsigned long long* out, float* o) {                                  \
        float x = threadIdx.x * 1e-3f;                                                         \
        asm volatile("v_mov_b32 v0, %0\n v_mov_b32 v1, %0\n v_mov_b32 v2, %0\n v_mov_b32 v3, %0\n v_mov_b32 v4, %0\n v_mov_b32 v5, %0\n v_mov_b32 v6, %0\n v_mov_b32 v7, %0\n v_mov_b32 v8, %0\n v_mov_b32 v9, %0" ::"v"(x) \
                     : "v0", "v1", "v2", "v3", "v4", "v5", "v6", "v7", "v8", "v9");            \
        unsigned long long t0 = __builtin_amdgcn_s_memtime();                                  \
        for (int i = 0; i < 64; ++i) asm volatile(BODY ::: "v0", "v1", "v2", "v3", "v4", "v5", "v6", "v7", "v8", "v9", "vcc"); \
        unsigned long long t1 = __builtin_amdgcn_s_memtime();                                  \
        float r;                                                                               \
        asm volatile("v_add_f32 %0, v0, v1" : "=v"(r));                                        \
        if ((threadIdx.x & 63) == 0) { out[2 * (threadIdx.x >> 6)] = t0; out[2 * (threadIdx.x >> 6) + 1] = t1; }                                       \
        if (r == 1234.5f) o[0] = r;                                                            \
    }
// 1 chain
KER(k_add1, R16("v_add_f32 v0, v0, v9\n"), 16)
KER(k_max1, R16("v_maximum3_f32 v0, v0, v9, v9\n"), 16)
KER(k_vmax1, R16("v_max_f32 v0, v0, v9\n"), 16)
KER(k_addmax1, R16("v_add_f32 v1, v0, v9\n v_maximum3_f32 v0, v1, v8, v8\n"), 32)
KER(k_dpp1, R16("v_mov_b32_dpp v0, v0 wave_shr:1 row_mask:0xf bank_mask:0xf\n"), 16)
KER(k_dppadd1, R16("v_mov_b32_dpp v1, v0 wave_shr:1 row_mask:0xf bank_mask:0xf\n v_add_f32 v0, v1, v9\n"), 32)
KER(k_dppaddf, R16("v_add_f32_dpp v0, v0, v9 wave_shr:1 row_mask:0xf bank_mask:0xf\n"), 16)
// 2 chains
KER(k_add2, R16("v_add_f32 v0, v0, v9\n v_add_f32 v1, v1, v9\n"), 32)
// 4 chains
KER(k_add4, R16("v_add_f32 v0, v0, v9\n v_add_f32 v1, v1, v9\n v_add_f32 v2, v2, v9\n v_add_f32 v3, v3, v9\n"), 64)
// 8 chains
KER(k_add8, R16("v_add_f32 v0, v0, v9\n v_add_f32 v1, v1, v9\n v_add_f32 v2, v2, v9\n v_add_f32 v3, v3, v9\n v_add_f32 v4, v4, v9\n v_add_f32 v5, v5, v9\n v_add_f32 v6, v6, v9\n v_add_f32 v7, v7, v9\n"), 128)
KER(k_max4, R16("v_maximum3_f32 v0, v0, v9, v9\n v_maximum3_f32 v1, v1, v9, v9\n v_maximum3_f32 v2, v2, v9, v9\n v_maximum3_f32 v3, v3, v9, v9\n"), 64)
KER(k_cmpaddc, R16("v_cmp_gt_f32 vcc, v0, v9\n v_addc_co_u32 v1, vcc, v1, v1, vcc\n"), 32)
KER(k_salu_dep, R16("s_add_u32 s20, s20, 1\n"), 16)
// fp64 / 64-bit integer chains (the column-0 routine's building blocks)
KER(k_f64add, R16("v_add_f64 v[0:1], v[0:1], v[8:9]\n"), 16)
KER(k_f64mul, R16("v_mul_f64 v[0:1], v[0:1], v[8:9]\n"), 16)
KER(k_f64rnd, R16("v_rndne_f64 v[0:1], v[0:1]\n"), 16)
KER(k_f64add4, R16("v_add_f64 v[0:1], v[0:1], v[8:9]\n v_add_f64 v[2:3], v[2:3], v[8:9]\n v_add_f64 v[4:5], v[4:5], v[8:9]\n v_add_f64 v[6:7], v[6:7], v[8:9]\n"), 64)
KER(k_u64add, R16("v_add_co_u32 v0, vcc, v0, v9\n v_addc_co_u32 v1, vcc, v1, v9, vcc\n"), 32)
KER(k_dpp64, R16("v_mov_b32_dpp v2, v0 row_shr:1 row_mask:0xf bank_mask:0xf bound_ctrl:1\n v_mov_b32_dpp v3, v1 row_shr:1 row_mask:0xf bank_mask:0xf bound_ctrl:1\n v_add_f64 v[0:1], v[0:1], v[2:3]\n"), 48)
KER(k_dppu64, R16("v_mov_b32_dpp v2, v0 row_shr:1 row_mask:0xf bank_mask:0xf bound_ctrl:1\n v_mov_b32_dpp v3, v1 row_shr:1 row_mask:0xf bank_mask:0xf bound_ctrl:1\n v_add_co_u32 v0, vcc, v0, v2\n v_addc_co_u32 v1, vcc, v1, v3, vcc\n"), 64)
KER(k_cvt64, R16("v_cvt_f64_f32 v[0:1], v2\n v_cvt_f32_f64 v2, v[0:1]\n"), 32)

int main() {
    unsigned long long* d;
    float* o;
    (void)hipMalloc(&d, 8 * 4096);
    (void)hipMalloc(&o, 64);
    struct { const char* n; void (*k)(unsigned long long*, float*); int per; } ks[] = {
        {"add chain", k_add1, 16}, {"maximum3 chain", k_max1, 16}, {"v_max chain", k_vmax1, 16},
        {"add->maximum3 chain", k_addmax1, 32}, {"dpp chain", k_dpp1, 16}, {"dpp->add chain", k_dppadd1, 32},
        {"add_dpp (fused) chain", k_dppaddf, 16}, {"add 2 chains", k_add2, 32}, {"add 4 chains", k_add4, 64},
        {"add 8 chains", k_add8, 128}, {"maximum3 4 chains", k_max4, 64}, {"cmp->addc pairs", k_cmpaddc, 32},
        {"salu chain", k_salu_dep, 16}, {"f64 add chain", k_f64add, 16}, {"f64 mul chain", k_f64mul, 16},
        {"f64 rndne chain", k_f64rnd, 16}, {"f64 add 4 chains", k_f64add4, 64}, {"u64 add (2 instr) chain", k_u64add, 32},
        {"dpp64 + f64 add (3 instr)", k_dpp64, 48}, {"dpp64 + u64 add (4 instr)", k_dppu64, 64},
        {"cvt f32->f64->f32 (2 instr)", k_cvt64, 32}};
    for (int wps : {1, 2, 4}) {
        printf("== %d wave(s) per SIMD (workgroup of %d waves on one CU)\n", wps, 4 * wps);
        for (auto& k : ks) {
            hipLaunchKernelGGL(k.k, dim3(1), dim3(64 * 4 * wps), 0, 0, d, o);
            (void)hipDeviceSynchronize();
            unsigned long long h[64];
            hipLaunchKernelGGL(k.k, dim3(1), dim3(64 * 4 * wps), 0, 0, d, o);
            (void)hipMemcpy(h, d, 8 * 2 * 4 * wps, hipMemcpyDeviceToHost);
            unsigned long long lo = ~0ull, hi = 0, sum = 0;
            for (int w = 0; w < 4 * wps; ++w) { lo = h[2*w] < lo ? h[2*w] : lo; hi = h[2*w+1] > hi ? h[2*w+1] : hi; sum += h[2*w+1] - h[2*w]; }
            double per_wave = (double)sum / (4 * wps) / (64.0 * k.per);
            double simd = (double)(hi - lo) / (64.0 * k.per * wps);  // cycles per instr per SIMD (all waves)
            printf("  %-26s wave-local %5.2f cyc/instr   span/SIMD %5.2f cyc/instr\n", k.n, per_wave, simd);
        }
    }
    return 0;
}
