#!/usr/bin/env python
"""Generates issue2.hip: per-step instruction mixes of the DP cell at 8 cells per lane
(development micro-benchmark; independent chains across cells, real dependence across steps)."""
C = 8
def cells(kind):
    L = []
    for k in range(C):  # s_k = cur_k + eb ; c_k = cur_{k-1} + et_k   (cur v16.., et v40.., s v48.., c v56.., w v64..)
        L.append(f"v_add_f32 v{48+k}, v{16+k}, v1")
        left = f"v{16+k-1}" if k else "v15"
        L.append(f"v_add_f32 v{56+k}, {left}, v{40+k}")
    for k in range(C):
        s, c, cur, w = f"v{48+k}", f"v{56+k}", f"v{16+k}", f"v{64+k}"
        if kind == "A":
            L += [f"v_cmp_gt_f32 vcc, {c}, {s}", f"v_addc_co_u32 {w}, vcc, {w}, {w}, vcc", f"v_maximum3_f32 {cur}, {s}, {c}, {c}"]
        elif kind == "B":
            L += [f"v_cmp_gt_f32 vcc, {c}, {s}", f"v_addc_co_u32 {w}, vcc, {w}, {w}, vcc", f"v_cndmask_b32 {cur}, {s}, {c}, vcc"]
        elif kind == "C":
            L += [f"v_max_f32 {cur}, {s}, {c}"]
        elif kind == "Cm3":
            L += [f"v_maximum3_f32 {cur}, {s}, {c}, {c}"]
        elif kind == "D":
            L += [f"v_sub_f32 v{72+k}, {s}, {c}", f"v_alignbit_b32 {w}, {w}, v{72+k}, 31", f"v_max_f32 {cur}, {s}, {c}"]
        elif kind == "E":
            p = f"s[{20+2*(k%4)}:{21+2*(k%4)}]"
            L += [f"v_cmp_gt_f32_e64 {p}, {c}, {s}", f"v_addc_co_u32_e64 {w}, {p}, {w}, {w}, {p}", f"v_cndmask_b32_e64 {cur}, {s}, {c}, {p}"]
        elif kind == "F":  # max first, then bit from max != s (sub-free)
            L += [f"v_max_f32 {cur}, {s}, {c}", f"v_cmp_gt_f32 vcc, {c}, {s}", f"v_addc_co_u32 {w}, vcc, {w}, {w}, vcc"]
        elif kind == "G":  # sub + alignbit bits, maximum3 (NaN-exact max)
            L += [f"v_sub_f32 v{72+k}, {s}, {c}", f"v_alignbit_b32 {w}, {w}, v{72+k}, 31", f"v_maximum3_f32 {cur}, {s}, {c}, {c}"]
    return L

def indep(op, n=16):
    return [op.format(i=16 + i) for i in range(n)]

K = {
    "add": indep("v_add_f32 v{i}, v1, v2"),
    "max": indep("v_max_f32 v{i}, v1, v2"),
    "maximum3": indep("v_maximum3_f32 v{i}, v1, v2, v2"),
    "cndmask_vcc": indep("v_cndmask_b32 v{i}, v1, v2, vcc"),
    "alignbit": indep("v_alignbit_b32 v{i}, v{i}, v2, 31"),
    "sub": indep("v_sub_f32 v{i}, v1, v2"),
    "cmp_vcc": indep("v_cmp_gt_f32 vcc, v{i}, v2"),
    "addc_vcc": indep("v_addc_co_u32 v{i}, vcc, v{i}, v{i}, vcc"),
    "pk_add": [f"v_pk_add_f32 v[{16+2*i}:{17+2*i}], v[2:3], v[4:5]" for i in range(16)],
    "dpp": indep("v_mov_b32_dpp v{i}, v1 wave_shr:1 row_mask:0xf bank_mask:0xf"),
    "ds_read_b32": [f"ds_read_b32 v{16+i}, v3 offset:{128*i}" for i in range(16)] + ["s_waitcnt lgkmcnt(0)"],
    "cellA(cur)": cells("A"), "cellB(cndmask)": cells("B"), "cellC(max only)": cells("C"),
    "cellCm3(maximum3 only)": cells("Cm3"), "cellD(sub,alignbit,max)": cells("D"),
    "cellE(e64 sgpr pairs)": cells("E"), "cellF(max,cmp,addc)": cells("F"), "cellG(sub,alignbit,maximum3)": cells("G"),
}
clob = ", ".join(f'"v{i}"' for i in range(1, 90)) + ', "vcc", "s20", "s21", "s22", "s23", "s24", "s25", "s26", "s27"'
out = ['#include <hip/hip_runtime.h>', '#include <stdio.h>', '#include <string.h>', '#include <stdlib.h>']
names = list(K)
for idx, n in enumerate(names):
    body = "\\n".join(K[n])
    out.append(f'__global__ void k{idx}(float* o, int iters) {{\n'
               f'  __shared__ float lds[4096]; lds[threadIdx.x] = threadIdx.x; __syncthreads();\n'
               f'  float x = threadIdx.x * 0.001f; unsigned a = (threadIdx.x % 32) * 4;\n'
               f'  asm volatile("v_mov_b32 v1, %0\\n v_mov_b32 v2, %0\\n v_mov_b32 v3, %1\\n v_mov_b32 v4, %0\\n v_mov_b32 v5, %0\\n v_mov_b32 v15, %0" :: "v"(x), "v"(a) : {clob});\n'
               f'  asm volatile("s_mov_b64 vcc, 0" ::: "vcc");\n'
               f'  for (int i = 0; i < iters; ++i) asm volatile("{body}" ::: {clob});\n'
               f'  float r; asm volatile("v_add_f32 %0, v16, v17" : "=v"(r));\n'
               f'  if (r == 12345.f) o[threadIdx.x] = r + lds[0];\n}}')
out.append('int main() { float* o; (void)hipMalloc(&o, 4096); const int iters = 1000;')
out.append('  struct K { const char* n; void (*k)(float*, int); int per; } ks[] = {')
for idx, n in enumerate(names):
    per = len([x for x in K[n] if not x.startswith("s_")])
    out.append(f'    {{"{n}", k{idx}, {per}}},')
out.append('  };')
out.append('''  for (int wps : {2, 4, 8}) { printf("== waves/SIMD %d (cycles per wave-instruction per SIMD; cell rows: per cell)\\n", wps);
    for (auto& k : ks) {
      hipLaunchKernelGGL(k.k, dim3(1024 * wps), dim3(64), 0, 0, o, 10);
      hipEvent_t a, b; (void)hipEventCreate(&a); (void)hipEventCreate(&b);
      (void)hipEventRecord(a); hipLaunchKernelGGL(k.k, dim3(1024 * wps), dim3(64), 0, 0, o, iters); (void)hipEventRecord(b);
      (void)hipEventSynchronize(b); float ms; (void)hipEventElapsedTime(&ms, a, b);
      double cyc = ms * 1e-3 * 2.4e9 / ((double)wps * iters);
      bool cell = strncmp(k.n, "cell", 4) == 0;
      printf("  %-30s %6.2f cyc/inst  %7.2f cyc/body%s\\n", k.n, cyc / k.per, cyc, cell ? "" : "");
      if (cell) printf("  %-30s %6.2f cyc/cell/SIMD\\n", "", cyc / 8);
    } }
  return 0; }''')
open("issue2.hip", "w").write("\n".join(out) + "\n")
