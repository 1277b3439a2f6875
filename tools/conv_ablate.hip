// Diagnostic: time the conv3x3 forward kernel with parts of its K loop removed
// (MODE bits, see conv3x3.hip) on one layer shape.  Build:
//   hipcc -O3 -std=c++17 --offload-arch=gfx950 tools/conv_ablate.hip -o tools/conv_ablate
// Run: tools/conv_ablate N H W CIN COUT [reps]
// Prints per-mode ms and TFLOP/s.  Not part of the product; outputs of modes != 0 are garbage.
#include "../enhanced-unet_amd/csrc/conv3x3.hip"
#include "../enhanced-unet_amd/csrc/capi.hip"

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <string>
#include <vector>

#define CK(x)                                                              \
  do {                                                                     \
    hipError_t e_ = (x);                                                   \
    if (e_ != hipSuccess) {                                                \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      exit(1);                                                             \
    }                                                                      \
  } while (0)

template <int MODE, bool DB = false, int NW = 4, bool SPEC = false, bool BDMA = false, bool PIPE = false>
static float run(const FwdArgs& a, dim3 grid, int reps) {
  const int lds = DB ? FWD_LDS_DB : FWD_LDS;
  allow_lds(conv3x3_fwd_kernel<bf16_t, MODE, DB, NW, SPEC, BDMA, 0, PIPE>, lds);
  conv3x3_fwd_kernel<bf16_t, MODE, DB, NW, SPEC, BDMA, 0, PIPE><<<grid, 64 * NW, lds>>>(a);
  CK(hipDeviceSynchronize());
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  CK(hipEventRecord(e0));
  for (int i = 0; i < reps; ++i) conv3x3_fwd_kernel<bf16_t, MODE, DB, NW, SPEC, BDMA, 0, PIPE><<<grid, 64 * NW, lds>>>(a);
  CK(hipEventRecord(e1));
  CK(hipEventSynchronize(e1));
  float ms = 0.f;
  CK(hipEventElapsedTime(&ms, e0, e1));
  return ms / reps;
}

template <int MODE>
static float run_wg(const WgArgs& a, dim3 grid, int reps) {
  allow_lds(conv3x3_wgrad_bf16_kernel<MODE>, WG_LDS);
  conv3x3_wgrad_bf16_kernel<MODE><<<grid, NTHR, WG_LDS>>>(a);
  CK(hipDeviceSynchronize());
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  CK(hipEventRecord(e0));
  for (int i = 0; i < reps; ++i) conv3x3_wgrad_bf16_kernel<MODE><<<grid, NTHR, WG_LDS>>>(a);
  CK(hipEventRecord(e1));
  CK(hipEventSynchronize(e1));
  float ms = 0.f;
  CK(hipEventElapsedTime(&ms, e0, e1));
  return ms / reps;
}

static int wgrad_main(int N, int H, int W, int cin, int cout, int reps) {
  const size_t nx = (size_t)N * H * W * cin, nd = (size_t)N * H * W * cout;
  std::vector<uint16_t> hx(nx), hd(nd);
  for (size_t i = 0; i < nx; ++i) hx[i] = 0x3c00 + (uint16_t)((i * 2654435761u) >> 24 & 0x7f);
  for (size_t i = 0; i < nd; ++i) hd[i] = 0x3c00 + (uint16_t)((i * 40503u) >> 8 & 0x7f);
  void *x, *dy;
  CK(hipMalloc(&x, nx * 2));
  CK(hipMalloc(&dy, nd * 2));
  CK(hipMemcpy(x, hx.data(), nx * 2, hipMemcpyHostToDevice));
  CK(hipMemcpy(dy, hd.data(), nd * 2, hipMemcpyHostToDevice));
  eunet_act dya = {dy, N, H, W, cout, cout, 0, EUNET_BF16};
  int ns = 0;
  eunet_conv3x3_wgrad_splits(&dya, cin, EUNET_BF16, &ns);
  float *dwp, *dbp;
  CK(hipMalloc(&dwp, (size_t)ns * cout * 9 * cin * 4));
  CK(hipMalloc(&dbp, (size_t)ns * cout * 4));
  WgArgs a;
  a.x = x; a.N = N; a.H = H; a.W = W; a.xct = cin; a.xco = 0; a.cin = cin;
  a.isc = nullptr; a.ish = nullptr; a.iss = 0; a.order = 0; a.phase = 0;
  a.dy = dy; a.dct = cout; a.dco = 0; a.cout = cout;
  a.dw = dwp; a.db = dbp;
  if (getenv("ABLATE_ISC") != nullptr) {  // BN+ReLU operand transform on (scale 1, shift 0)
    std::vector<float> one(cin, 1.f), zero(cin, 0.f);
    float *sc, *sh;
    CK(hipMalloc(&sc, cin * 4));
    CK(hipMalloc(&sh, cin * 4));
    CK(hipMemcpy(sc, one.data(), cin * 4, hipMemcpyHostToDevice));
    CK(hipMemcpy(sh, zero.data(), cin * 4, hipMemcpyHostToDevice));
    a.isc = sc;
    a.ish = sh;
  }
  a.tx = cdiv(W, TW); a.ty = cdiv(H, TH); a.ntiles = N * a.tx * a.ty;
  a.per_split = cdiv(a.ntiles, ns);
  a.nsplit = ns;
  dim3 grid(ns * cdiv(cout, 64) * cdiv(cin, KCW));
  const double flop = 2.0 * 9 * cin * cout * (double)N * H * W;
  const float t0 = run_wg<0>(a, grid, reps), t1 = run_wg<1>(a, grid, reps), t2 = run_wg<2>(a, grid, reps),
              t3 = run_wg<3>(a, grid, reps);
  printf("{\"wgrad_shape\": [%d, %d, %d, %d, %d], \"blocks\": %u, \"splits\": %d", N, H, W, cin, cout, grid.x, ns);
  const char* nm[] = {"full", "stage_once", "no_mfma", "lds_only"};
  const float ts[] = {t0, t1, t2, t3};
  for (int i = 0; i < 4; ++i) printf(", \"%s_ms\": %.4f, \"%s_tf\": %.1f", nm[i], ts[i], nm[i], flop / ts[i] / 1e9);
  printf("}\n");
  return 0;
}

template <int ABL>
static float run_k64(const FwdArgs& a, int reps) {
  const int ncob = a.cout_pad / BN;
  const dim3 grid(std::max(1, std::min(a.ntiles, 256 / ncob)) * ncob);
  allow_lds(conv3x3_k64_kernel<ABL>, K64_LDS);
  conv3x3_k64_kernel<ABL><<<grid, K64_T, K64_LDS>>>(a);
  CK(hipDeviceSynchronize());
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  CK(hipEventRecord(e0));
  for (int i = 0; i < reps; ++i) conv3x3_k64_kernel<ABL><<<grid, K64_T, K64_LDS>>>(a);
  CK(hipEventRecord(e1));
  CK(hipEventSynchronize(e1));
  float ms = 0.f;
  CK(hipEventElapsedTime(&ms, e0, e1));
  return ms / reps;
}

int main(int argc, char** argv) {
  if (argc >= 7 && std::string(argv[1]) == "wgrad")
    return wgrad_main(atoi(argv[2]), atoi(argv[3]), atoi(argv[4]), atoi(argv[5]), atoi(argv[6]),
                      argc > 7 ? atoi(argv[7]) : 10);
  if (argc < 6) {
    fprintf(stderr, "usage: %s N H W CIN COUT [reps]\n", argv[0]);
    return 2;
  }
  const int N = atoi(argv[1]), H = atoi(argv[2]), W = atoi(argv[3]), cin = atoi(argv[4]), cout = atoi(argv[5]);
  const int reps = argc > 6 ? atoi(argv[6]) : 10;
  if (N <= 0 || H <= 0 || W <= 0 || cin % 32 || cout % 64 || (long long)N * H * W * (cin + cout) > (1ll << 31)) {
    fprintf(stderr, "bad shape\n");
    return 2;
  }
  const size_t nx = (size_t)N * H * W * cin, ny = (size_t)N * H * W * cout;
  std::vector<uint16_t> hx(nx);
  for (size_t i = 0; i < nx; ++i) hx[i] = 0x3c00 + (uint16_t)((i * 2654435761u) >> 24 & 0x7f);  // ~[1,2)
  std::vector<float> hw((size_t)cout * cin * 9);
  for (size_t i = 0; i < hw.size(); ++i) hw[i] = ((int)((i * 40503u) & 255) - 128) / 4096.f;
  void *x, *y, *wp;
  float *w, *stats;
  CK(hipMalloc(&x, nx * 2));
  CK(hipMalloc(&y, ny * 2));
  CK(hipMalloc(&w, hw.size() * 4));
  size_t wpb = 0;
  eunet_conv3x3_packed_bytes(cout, cin, EUNET_BF16, &wpb);
  CK(hipMalloc(&wp, wpb));
  CK(hipMemcpy(x, hx.data(), nx * 2, hipMemcpyHostToDevice));
  CK(hipMemcpy(w, hw.data(), hw.size() * 4, hipMemcpyHostToDevice));
  if (eunet_conv3x3_pack(w, cout, cin, 0, wp, EUNET_BF16, nullptr)) {
    fprintf(stderr, "pack: %s\n", eunet_last_error());
    return 1;
  }
  FwdArgs a;
  a.x = x; a.N = N; a.H = H; a.W = W; a.xct = cin; a.xco = 0; a.cin = cin;
  a.isc = nullptr; a.ish = nullptr; a.iss = 0;
  a.wp = wp; a.cout_pad = cout; a.nkc = cin / 32;
  a.bias = nullptr;
  a.y = y; a.yct = cout; a.yco = 0; a.cout = cout;
  a.tx = cdiv(W, FTW); a.ty = cdiv(H, FTH); a.ntiles = N * a.tx * a.ty;
  a.by = nullptr; a.byct = 0; a.byco = 0;
  a.bmean = a.bistd = a.bgam = a.bbet = nullptr; a.bpart = nullptr; a.gsc = nullptr; a.order = 0; a.phase = 0; a.pro1 = 0;
  CK(hipMalloc(&stats, (size_t)a.ntiles * (2 * cout + 1) * 4));
  a.stats = stats;
  if (getenv("ABLATE_ISC") != nullptr) {  // BN+ReLU operand transform on (scale 1, shift 0)
    std::vector<float> one(cin, 1.f), zero(cin, 0.f);
    float *sc, *sh;
    CK(hipMalloc(&sc, cin * 4));
    CK(hipMalloc(&sh, cin * 4));
    CK(hipMemcpy(sc, one.data(), cin * 4, hipMemcpyHostToDevice));
    CK(hipMemcpy(sh, zero.data(), cin * 4, hipMemcpyHostToDevice));
    a.isc = sc;
    a.ish = sh;
  }
  dim3 grid(a.ntiles * (cout / BN));
  const double flop = 2.0 * 9 * cin * cout * (double)N * H * W;
  if (getenv("ABLATE_K64") != nullptr && cin == 64) {  // persistent Cin=64 kernel ablation
    const char* nm[] = {"k64_full", "k64_stage_once", "k64_no_epi", "k64_mfma_lds_only", "k64_no_mfma",
                        "k64_no_mfma_no_epi", "k64_no_store", "k64_no_stats"};
    const float ts0 = run_k64<0>(a, reps);
    float* st = a.stats;
    a.stats = nullptr;
    const float tns = run_k64<0>(a, reps);
    a.stats = st;
    const float ts[] = {ts0, run_k64<1>(a, reps), run_k64<2>(a, reps), run_k64<3>(a, reps),
                        run_k64<4>(a, reps), run_k64<6>(a, reps), run_k64<8>(a, reps), tns};
    printf("{\"shape\": [%d, %d, %d, %d, %d]", N, H, W, cin, cout);
    for (int i = 0; i < 8; ++i) printf(", \"%s_ms\": %.4f, \"%s_tf\": %.1f", nm[i], ts[i], nm[i], flop / ts[i] / 1e9);
    printf("}\n");
    return 0;
  }
  const float t0 = run<0>(a, grid, reps), t1 = run<1>(a, grid, reps), t2 = run<2>(a, grid, reps);
  const float t4 = run<4>(a, grid, reps), t5 = run<5>(a, grid, reps), t8 = run<8>(a, grid, reps);
  const float tdb = run<0, true, 8>(a, grid, reps), tdb5 = run<5, true, 8>(a, grid, reps);
  const float t8w = run<0, false, 8>(a, grid, reps);
  const float tsp = run<0, true, 8, true>(a, grid, reps), tsp5 = run<5, true, 8, true>(a, grid, reps);
  const float tdb4 = run<0, true, 4>(a, grid, reps);
  const float td16 = run<16>(a, grid, reps), td32 = run<32>(a, grid, reps);
  const float tp4 = run<0, true, 4, false, false, true>(a, grid, reps);
  const float tp4m = run<5, true, 4, false, false, true>(a, grid, reps);
  const float tp2 = run<0, false, 4, false, false, true>(a, grid, reps);
  const float tbd8 = run<0, true, 8, false, true>(a, grid, reps), tbd4 = run<0, true, 4, false, true>(a, grid, reps);
  printf("{\"shape\": [%d, %d, %d, %d, %d], \"blocks\": %d", N, H, W, cin, cout, a.ntiles * cout / BN);
  const char* nm[] = {"full", "no_gload", "no_mfma", "no_ldsread", "mfma_only", "tile_fastest", "db8_full",
                      "db8_mfma_only", "w8_2blk_full", "spec_full", "spec_mfma_only", "db4_full", "db8_bdma",
                      "db4_bdma", "delay2k", "delay5k", "db4_pipe",
                      "db4_pipe_mfma_only", "pipe_2blk"};
  const float ts[] = {t0, t1, t2, t4, t5, t8, tdb, tdb5, t8w, tsp, tsp5, tdb4, tbd8, tbd4, td16, td32, tp4, tp4m, tp2};
  for (int i = 0; i < 19; ++i) printf(", \"%s_ms\": %.4f, \"%s_tf\": %.1f", nm[i], ts[i], nm[i], flop / ts[i] / 1e9);
  printf("}\n");
  return 0;
}
