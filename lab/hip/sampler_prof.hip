// Lab driver: phase timestamps of the decode sampler (csrc/sampling.hip built with
// MP_SAMPLE_PROF), 64 rows x 32000 vocab, reference CLI parameters (T 1, top-p 0.92, top-k 50,
// repetition penalty 1.5, 10-id history).  Prints per-phase cycles (median over rows) and the
// top-k candidate count.
//   hipcc -O3 --offload-arch=gfx950 -DMP_SAMPLE_PROF -I <pkg>/ops/csrc scripts/sampler_prof.hip -o _lab/sampler_prof
#include "sampling.hip"
#include <algorithm>
#include <cstring>
#include <cstdio>
#include <random>
#include <vector>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP %s @%d\n", hipGetErrorString(e_), __LINE__); return 1; } } while (0)

static unsigned short f2bf_h(float f) { unsigned u; std::memcpy(&u, &f, 4); return (unsigned short)((u + 0x7fff + ((u >> 16) & 1)) >> 16); }

int main(int argc, char** argv) {
  const int R = 64, V = argc > 1 ? atoi(argv[1]) : 32000, CAP = 50, H = 10;
  std::mt19937 g(5);
  std::normal_distribution<float> nd(0.f, 3.f);
  std::vector<unsigned short> lg((size_t)R * V);
  for (auto& v : lg) v = f2bf_h(nd(g));
  std::vector<float> temps(R, 1.f), tps(R, 0.92f), rps(R, 1.5f);
  std::vector<int32_t> tks(R, 50), rec((size_t)R * CAP), rlen(R, H);
  for (auto& v : rec) v = g() % V;
  std::vector<int64_t> seeds(R);
  for (int i = 0; i < R; ++i) seeds[i] = i;
  void *d_lg, *d_t, *d_tp, *d_tk, *d_rp, *d_rec, *d_rl, *d_seed, *d_ws, *d_out;
  CK(hipMalloc(&d_lg, lg.size() * 2)); CK(hipMalloc(&d_t, R * 4)); CK(hipMalloc(&d_tp, R * 4));
  CK(hipMalloc(&d_tk, R * 4)); CK(hipMalloc(&d_rp, R * 4)); CK(hipMalloc(&d_rec, rec.size() * 4));
  CK(hipMalloc(&d_rl, R * 4)); CK(hipMalloc(&d_seed, R * 8)); CK(hipMalloc(&d_ws, (size_t)R * V * 4));
  CK(hipMalloc(&d_out, R * 8));
  CK(hipMemcpy(d_lg, lg.data(), lg.size() * 2, hipMemcpyHostToDevice));
  CK(hipMemcpy(d_t, temps.data(), R * 4, hipMemcpyHostToDevice));
  CK(hipMemcpy(d_tp, tps.data(), R * 4, hipMemcpyHostToDevice));
  CK(hipMemcpy(d_tk, tks.data(), R * 4, hipMemcpyHostToDevice));
  CK(hipMemcpy(d_rp, rps.data(), R * 4, hipMemcpyHostToDevice));
  CK(hipMemcpy(d_rec, rec.data(), rec.size() * 4, hipMemcpyHostToDevice));
  CK(hipMemcpy(d_seed, seeds.data(), R * 8, hipMemcpyHostToDevice));
  std::vector<unsigned long long> prof(1024 * 16);
  for (int it = 0; it < 5; ++it) {
    CK(hipMemcpy(d_rl, rlen.data(), R * 4, hipMemcpyHostToDevice));
    int rc = mp_sample(d_lg, V, R, V, (float*)d_t, (float*)d_tp, (int32_t*)d_tk, (float*)d_rp, (int32_t*)d_rec, CAP,
                       (int32_t*)d_rl, (int64_t*)d_seed, (float*)d_ws, (int64_t*)d_out, 1, 0);
    if (rc) { printf("launch rc %d\n", rc); return 1; }
    CK(hipDeviceSynchronize());
  }
  CK(hipMemcpyFromSymbol(prof.data(), HIP_SYMBOL(mp::mp_sprof), prof.size() * 8));
  const char* names[] = {"copy+hist", "penalty", "max", "expsum", "tau", "collect", "rank", "write_p", "scans+draw", "append"};
  for (int ph = 0; ph < 10; ++ph) {
    std::vector<long long> d;
    for (int r = 0; r < R; ++r) d.push_back((long long)(prof[r * 16 + ph + 1] - prof[r * 16 + ph]));
    std::sort(d.begin(), d.end());
    printf("%-12s median %7lld cycles  max %7lld\n", names[ph], d[R / 2], d.back());
  }
  std::vector<long long> tot, cnt;
  for (int r = 0; r < R; ++r) { tot.push_back((long long)(prof[r * 16 + 10] - prof[r * 16])); cnt.push_back((long long)prof[r * 16 + 15]); }
  std::sort(tot.begin(), tot.end()); std::sort(cnt.begin(), cnt.end());
  printf("total        median %7lld cycles; candidates median %lld max %lld\n", tot[R / 2], cnt[R / 2], cnt.back());
  return 0;
}
