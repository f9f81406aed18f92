// Which hipBLASLt epilogue GEMMs does this gfx950 install have kernels for?  Asks the heuristic
// (no launch) for every combination the fused dense layers could use and prints one JSON line per
// combination: dtype x epilogue x bias dtype x aux dtype x transposes x shape.
// Build: hipcc -O2 -std=c++17 tools/lt_probe.cpp -lhipblaslt -o /tmp/lt_probe  (host only)
#include <hip/hip_runtime.h>
#include <hipblaslt/hipblaslt.h>

#include <cstdio>
#include <vector>

static const char* tname(hipDataType t) {
  switch (t) {
    case HIP_R_16BF: return "bf16";
    case HIP_R_16F: return "f16";
    case HIP_R_32F: return "f32";
    default: return "?";
  }
}

int main() {
  hipblasLtHandle_t h;
  if (hipblasLtCreate(&h) != HIPBLAS_STATUS_SUCCESS) {
    printf("{\"error\": \"hipblasLtCreate\"}\n");
    return 1;
  }
  struct Epi { hipblasLtEpilogue_t e; const char* name; bool aux; bool bias; };
  const Epi epis[] = {{HIPBLASLT_EPILOGUE_BIAS, "BIAS", false, true},
                      {HIPBLASLT_EPILOGUE_GELU_BIAS, "GELU_BIAS", false, true},
                      {HIPBLASLT_EPILOGUE_GELU_AUX_BIAS, "GELU_AUX_BIAS", true, true},
                      {HIPBLASLT_EPILOGUE_GELU_AUX, "GELU_AUX", true, false},
                      {HIPBLASLT_EPILOGUE_DGELU_BGRAD, "DGELU_BGRAD", true, true},
                      {HIPBLASLT_EPILOGUE_DGELU, "DGELU", true, false},
                      {HIPBLASLT_EPILOGUE_BGRADB, "BGRADB", false, true},
                      {HIPBLASLT_EPILOGUE_BGRADA, "BGRADA", false, true}};
  const hipDataType dts[] = {HIP_R_16BF, HIP_R_16F};
  struct Shape { long m, n, k; };
  const Shape shapes[] = {{4096, 16384, 1024}, {1024, 16384, 4096}, {2048, 1000, 512}};
  for (hipDataType dt : dts)
    for (const Epi& ep : epis)
      for (int bt = 0; bt < 2; ++bt)
        for (int at = 0; at < 3; ++at)
          for (int ta = 0; ta < 2; ++ta)
            for (int tb = 0; tb < 2; ++tb)
              for (const Shape& s : shapes) {
                if (!ep.aux && at != 0) continue;
                if (!ep.bias && bt != 0) continue;
                hipblasLtMatmulDesc_t d;
                hipblasLtMatmulDescCreate(&d, HIPBLAS_COMPUTE_32F, HIP_R_32F);
                int32_t opa = ta ? HIPBLAS_OP_T : HIPBLAS_OP_N, opb = tb ? HIPBLAS_OP_T : HIPBLAS_OP_N;
                hipblasLtMatmulDescSetAttribute(d, HIPBLASLT_MATMUL_DESC_TRANSA, &opa, sizeof(opa));
                hipblasLtMatmulDescSetAttribute(d, HIPBLASLT_MATMUL_DESC_TRANSB, &opb, sizeof(opb));
                hipblasLtMatmulDescSetAttribute(d, HIPBLASLT_MATMUL_DESC_EPILOGUE, &ep.e, sizeof(ep.e));
                const hipDataType btype = bt ? HIP_R_32F : dt;
                if (ep.bias) {
                  int32_t b = btype;
                  hipblasLtMatmulDescSetAttribute(d, HIPBLASLT_MATMUL_DESC_BIAS_DATA_TYPE, &b, sizeof(b));
                  void* fake = (void*)0x100000;
                  hipblasLtMatmulDescSetAttribute(d, HIPBLASLT_MATMUL_DESC_BIAS_POINTER, &fake, sizeof(fake));
                }
                hipDataType atype = dt;
                if (ep.aux) {
                  void* fake = (void*)0x200000;
                  hipblasLtMatmulDescSetAttribute(d, HIPBLASLT_MATMUL_DESC_EPILOGUE_AUX_POINTER, &fake, sizeof(fake));
                  int64_t ld = s.m;
                  hipblasLtMatmulDescSetAttribute(d, HIPBLASLT_MATMUL_DESC_EPILOGUE_AUX_LD, &ld, sizeof(ld));
                  if (at > 0) {
                    atype = at == 1 ? dt : HIP_R_32F;
                    int32_t a = atype;
                    hipblasLtMatmulDescSetAttribute(d, HIPBLASLT_MATMUL_DESC_EPILOGUE_AUX_DATA_TYPE, &a, sizeof(a));
                  }
                }
                hipblasLtMatrixLayout_t la, lb, lc;
                hipblasLtMatrixLayoutCreate(&la, dt, ta ? s.k : s.m, ta ? s.m : s.k, ta ? s.k : s.m);
                hipblasLtMatrixLayoutCreate(&lb, dt, tb ? s.n : s.k, tb ? s.k : s.n, tb ? s.n : s.k);
                hipblasLtMatrixLayoutCreate(&lc, dt, s.m, s.n, s.m);
                hipblasLtMatmulPreference_t pref;
                hipblasLtMatmulPreferenceCreate(&pref);
                uint64_t ws = 32ull << 20;
                hipblasLtMatmulPreferenceSetAttribute(pref, HIPBLASLT_MATMUL_PREF_MAX_WORKSPACE_BYTES, &ws, sizeof(ws));
                hipblasLtMatmulHeuristicResult_t res[4];
                int found = 0;
                hipblasStatus_t st = hipblasLtMatmulAlgoGetHeuristic(h, d, la, lb, lc, lc, pref, 4, res, &found);
                printf("{\"dtype\": \"%s\", \"epilogue\": \"%s\", \"bias\": \"%s\", \"aux\": \"%s\", \"ta\": %d, \"tb\": %d, "
                       "\"m\": %ld, \"n\": %ld, \"k\": %ld, \"status\": %d, \"found\": %d}\n",
                       tname(dt), ep.name, ep.bias ? tname(btype) : "-", ep.aux ? (at ? tname(atype) : "default") : "-",
                       ta, tb, s.m, s.n, s.k, (int)st, found);
                hipblasLtMatmulPreferenceDestroy(pref);
                hipblasLtMatrixLayoutDestroy(la);
                hipblasLtMatrixLayoutDestroy(lb);
                hipblasLtMatrixLayoutDestroy(lc);
                hipblasLtMatmulDescDestroy(d);
              }
  hipblasLtDestroy(h);
  return 0;
}
