// tail_bench.hip -- the persistent K = 7 kernels' tail (VERDICT r05 "Next round" #1): per-wave
// stamps and paired timing of the static group walk against the group queue (acs_persist.hpp
// GroupQueue), soft (viterbi_soft_persist, the headline) and hard (viterbi_hard_persist, config 4),
// on the headline's batch: 104 frames x 25,000 blocks = 2.6 M blocks of blen 40 (T = 46).
//
// Error counting on (info bytes given), as on the bench path. Then the K = 9 persistent kernels
// (acs_wide.hpp x86-idiom code, acs_multi2.hpp true parity) at the K = 9 bench batch, 32 frames.
//   tail_bench [outdir]   stamps -> outdir/stamps_{soft,hard}_{static,queue}.csv (one row per wave)
//
// Every schedule's output bytes are compared with the static walk's (the queue must decode every
// group exactly once). Build: hipcc -O3 -std=c++20 --offload-arch=gfx950 -fno-slp-vectorize
//   -I../include -I../convolutional-codes_amd/csrc tail_bench.hip -o tail_bench
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <map>
#include <string>
#include <tuple>
#include <vector>

#include "acs_multi2.hpp"
#include "acs_persist.hpp"
#include "acs_wide.hpp"
#include "reg_codes.hpp"

using namespace ccv;
constexpr CodeSpec kK7Ref{2, 7, {0xF200000000000000ull, 0xB600000000000000ull, 0, 0, 0, 0, 0, 0}, GEN_REF_X86};

#define CHECK(x)                                                              \
  do {                                                                        \
    hipError_t e = (x);                                                       \
    if (e != hipSuccess) {                                                    \
      fprintf(stderr, "%s: %s (line %d)\n", #x, hipGetErrorString(e), __LINE__); \
      exit(1);                                                                \
    }                                                                         \
  } while (0)

__global__ void fill_soft(float* p, size_t n) {
  for (size_t i = (size_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (size_t)gridDim.x * 256) {
    uint32_t x = (uint32_t)i * 0x9E3779B9u ^ (uint32_t)(i >> 32);
    x ^= x >> 15; x *= 0x85EBCA6Bu; x ^= x >> 13; x *= 0xC2B2AE35u; x ^= x >> 16;
    p[i] = (float)(x >> 8) * (1.0f / 16777216.0f) * 3.0f;
  }
}
__global__ void fill_hard(uint8_t* p, size_t n) {
  for (size_t i = (size_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (size_t)gridDim.x * 256) {
    uint32_t x = (uint32_t)i * 0x9E3779B9u;
    x ^= x >> 15; x *= 0x85EBCA6Bu; x ^= x >> 13;
    p[i] = (uint8_t)(x >> 29);   // BSC symbols (the kernel masks to n bits)
  }
}

using Kern = void (*)(RegArgs, int);

struct Setup {
  RegArgs a;
  int ngroups, grid;
};

int grid_of(Kern k, int ngroups) {
  int per_cu = 0, cus = 0;
  CHECK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, k, 64, 0));
  CHECK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
  if (per_cu >= 4) per_cu -= per_cu % 4;
  return std::min(per_cu * cus, ngroups);
}

float sustained(Kern k, const Setup& s, int n) {
  const int grid = grid_of(k, s.ngroups);
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0));
  CHECK(hipEventCreate(&e1));
  CHECK(hipEventRecord(e0, 0));
  for (int i = 0; i < n; ++i) hipLaunchKernelGGL(k, dim3(grid), dim3(64), 0, 0, s.a, s.ngroups);
  CHECK(hipEventRecord(e1, 0));
  CHECK(hipEventSynchronize(e1));
  float ms = 0;
  CHECK(hipEventElapsedTime(&ms, e0, e1));
  CHECK(hipEventDestroy(e0));
  CHECK(hipEventDestroy(e1));
  return ms / n;
}

// One stamped launch after a warm clock; per-wave table + summary.
void stamp_run(const char* tag, Kern k, Setup s, uint32_t* d_stamps, const std::string& outdir) {
  const int grid = grid_of(k, s.ngroups);
  s.a.stamps = d_stamps;
  for (int i = 0; i < 30; ++i) hipLaunchKernelGGL(k, dim3(grid), dim3(64), 0, 0, s.a, s.ngroups);
  CHECK(hipDeviceSynchronize());
  std::vector<uint32_t> h((size_t)grid * kStampWords);
  CHECK(hipMemcpy(h.data(), d_stamps, h.size() * 4, hipMemcpyDeviceToHost));
  uint64_t t0 = ~0ull, t1 = 0;
  for (int w = 0; w < grid; ++w) {
    const uint32_t* r = &h[(size_t)w * kStampWords];
    t0 = std::min(t0, (uint64_t)r[0] | (uint64_t)r[1] << 32);
    t1 = std::max(t1, (uint64_t)r[2] | (uint64_t)r[3] << 32);
  }
  const double span = (double)(t1 - t0);
  std::vector<double> life, ends, starts;
  std::map<int, std::vector<double>> end_by_xcc, end_by_slot;
  std::map<uint32_t, int> groups_hist;
  uint32_t steals = 0;
  FILE* f = fopen((outdir + "/stamps_" + tag + ".csv").c_str(), "w");
  if (f) fprintf(f, "wave,start_us,end_us,xcc,se,cu,simd,wave_slot,groups,steals\n");
  // SIMD occupancy order: waves on the same SIMD ranked by start time (0 = oldest)
  std::map<std::tuple<int, int, int, int>, std::vector<std::pair<double, int>>> per_simd;
  for (int w = 0; w < grid; ++w) {
    const uint32_t* r = &h[(size_t)w * kStampWords];
    const double st = (double)(((uint64_t)r[0] | (uint64_t)r[1] << 32) - t0) / 100.0;   // us (100 MHz)
    const double en = (double)(((uint64_t)r[2] | (uint64_t)r[3] << 32) - t0) / 100.0;
    const uint32_t hw = r[4];
    const int simd = (hw >> 4) & 3, cu = (hw >> 8) & 15, se = (hw >> 13) & 7, slot = hw & 15;
    const int xcc = (int)(r[5] & 15);
    life.push_back(en - st);
    ends.push_back(en);
    starts.push_back(st);
    end_by_xcc[xcc].push_back(en);
    groups_hist[r[6]]++;
    steals += r[7];
    per_simd[{xcc, se, cu, simd}].push_back({st, w});
    if (f) fprintf(f, "%d,%.3f,%.3f,%d,%d,%d,%d,%d,%u,%u\n", w, st, en, xcc, se, cu, simd, slot, r[6], r[7]);
  }
  if (f) fclose(f);
  for (auto& [key, v] : per_simd) {
    std::sort(v.begin(), v.end());
    for (size_t i = 0; i < v.size(); ++i) end_by_slot[(int)i].push_back(ends[v[i].second]);
  }
  double lsum = 0;
  for (double l : life) lsum += l;
  std::sort(ends.begin(), ends.end());
  std::sort(starts.begin(), starts.end());
  auto q = [&](const std::vector<double>& v, double p) { return v[(size_t)(p * (v.size() - 1))]; };
  printf("[%s] waves %d  span %.1f us  lifetime ratio %.3f  start max %.1f us  end q0 %.1f q10 %.1f q50 %.1f q90 %.1f q100 %.1f us  steals %u\n",
         tag, grid, span / 100.0, lsum / grid / (span / 100.0), starts.back(), ends.front(), q(ends, 0.1),
         q(ends, 0.5), q(ends, 0.9), ends.back(), steals);
  printf("[%s] groups per wave:", tag);
  for (auto& [g, n] : groups_hist) printf(" %u:%d", g, n);
  printf("\n[%s] mean end per XCC:", tag);
  for (auto& [x, v] : end_by_xcc) {
    double m = 0;
    for (double e : v) m += e;
    printf(" %d:%.1f", x, m / v.size());
  }
  printf("\n[%s] mean end by age rank on its SIMD (0 = oldest):", tag);
  for (auto& [x, v] : end_by_slot) {
    double m = 0;
    for (double e : v) m += e;
    printf(" %d:%.1f(n=%zu)", x, m / v.size(), v.size());
  }
  printf("\n");
}

int main(int argc, char** argv) {
  const std::string outdir = argc > 1 ? argv[1] : ".";
  const int nb = 2600000, T = 46, blen = 40, ng = nb / 64;
  float* d_soft;
  uint8_t *d_hard, *d_out_a, *d_out_b;
  uint32_t *d_queue, *d_stamps;
  CHECK(hipMalloc(&d_soft, (size_t)nb * T * 16));
  CHECK(hipMalloc(&d_hard, (size_t)nb * T));
  CHECK(hipMalloc(&d_out_a, (size_t)nb * 8));
  CHECK(hipMalloc(&d_out_b, (size_t)nb * 8));
  CHECK(hipMalloc(&d_queue, kQueueWords * 4));
  uint8_t* d_info;   // transmitted info bytes: the bench path counts errors (5 bytes per block)
  unsigned long long* d_err;
  CHECK(hipMalloc(&d_info, (size_t)nb * 5));
  CHECK(hipMalloc(&d_err, 8));
  CHECK(hipMemset(d_err, 0, 8));
  CHECK(hipMalloc(&d_stamps, 65536 * kStampWords * 4));
  CHECK(hipMemset(d_queue, 0, kQueueWords * 4));
  hipLaunchKernelGGL(fill_soft, dim3(8192), dim3(256), 0, 0, d_soft, (size_t)nb * T * 4);
  hipLaunchKernelGGL(fill_hard, dim3(8192), dim3(256), 0, 0, d_hard, (size_t)nb * T);
  hipLaunchKernelGGL(fill_hard, dim3(8192), dim3(256), 0, 0, d_info, (size_t)nb * 5);
  CHECK(hipDeviceSynchronize());

  Setup soft{}, hard{};
  soft.a.in = d_soft;
  soft.a.T = T;
  soft.a.nblocks = nb;
  soft.a.blen = blen;
  soft.a.queue = d_queue;
  soft.a.info = d_info;
  soft.a.err = d_err;
  soft.ngroups = ng;
  hard = soft;
  hard.a.in = d_hard;

  constexpr int IF = kPersistInfoFirst, QU = kPersistQueue, ST = kPersistStamp, H1 = kPersistQueueHop1,
                H7 = kPersistQueueHop7;
  const Kern ks = viterbi_soft_persist<kK7Ref, 40, 0>, kq0 = viterbi_soft_persist<kK7Ref, 40, QU>,
             kq1 = viterbi_soft_persist<kK7Ref, 40, QU | H1>, kq7 = viterbi_soft_persist<kK7Ref, 40, QU | H7>;
  const Kern kss = viterbi_soft_persist<kK7Ref, 40, ST>, kq0s = viterbi_soft_persist<kK7Ref, 40, QU | ST>,
             kq1s = viterbi_soft_persist<kK7Ref, 40, QU | H1 | ST>;
  const Kern hs = viterbi_hard_persist<kK7Ref, 40, 3, 0>, hf = viterbi_hard_persist<kK7Ref, 40, 3, IF>,
             hq0 = viterbi_hard_persist<kK7Ref, 40, 3, QU | IF>, hq1 = viterbi_hard_persist<kK7Ref, 40, 3, QU | IF | H1>,
             hq7 = viterbi_hard_persist<kK7Ref, 40, 3, QU | IF | H7>;
  const Kern hss = viterbi_hard_persist<kK7Ref, 40, 3, ST>,
             hq0s = viterbi_hard_persist<kK7Ref, 40, 3, QU | IF | ST>,
             hq1s = viterbi_hard_persist<kK7Ref, 40, 3, QU | IF | H1 | ST>;

  // exactness: every schedule writes the static walk's bytes
  int bad = 0;
  auto compare = [&](const char* name, Kern ref, Kern k, Setup s, int n = nb) {
    for (uint8_t* o : {d_out_a, d_out_b}) CHECK(hipMemset(o, 0xA5, (size_t)nb * 8));
    const int g = (n + 63) / 64;
    s.a.nblocks = n;
    s.a.out = d_out_a;
    s.a.stamps = d_stamps;
    hipLaunchKernelGGL(ref, dim3(grid_of(ref, g)), dim3(64), 0, 0, s.a, g);
    s.a.out = d_out_b;
    for (int rep = 0; rep < 3; ++rep)   // repeated: the queue must have reset itself
      hipLaunchKernelGGL(k, dim3(grid_of(k, g)), dim3(64), 0, 0, s.a, g);
    CHECK(hipDeviceSynchronize());
    std::vector<uint8_t> x((size_t)nb * 8), y((size_t)nb * 8);
    CHECK(hipMemcpy(x.data(), d_out_a, x.size(), hipMemcpyDeviceToHost));
    CHECK(hipMemcpy(y.data(), d_out_b, y.size(), hipMemcpyDeviceToHost));
    std::vector<uint32_t> qw(kQueueWords);
    CHECK(hipMemcpy(qw.data(), d_queue, qw.size() * 4, hipMemcpyDeviceToHost));
    bool zero = true;
    for (uint32_t v : qw) zero = zero && v == 0;
    const bool same = x == y;
    printf("%s (%d groups): outputs %s the static walk's; queue words after the launches %s\n", name, g,
           same ? "identical to" : "DIFFER from", zero ? "all zero" : "NOT ZERO");
    bad += !same || !zero;
  };
  soft.a.out = d_out_a;
  hard.a.out = d_out_a;
  for (int n : {nb, 64 * 5, 64 * 9 + 17, 64 * 3000 + 1}) {   // all labels; fewer waves than labels; ragged
    compare("soft queue hop0", ks, kq0, soft, n);
    compare("soft queue hop1", ks, kq1, soft, n);
    compare("soft queue hop7", ks, kq7, soft, n);
    if (n % 64 == 0) {   // the hard kernel stages whole groups (the host sends a partial one elsewhere)
      compare("hard queue hop0", hs, hq0, hard, n);
      compare("hard queue hop1", hs, hq1, hard, n);
      compare("hard queue hop7", hs, hq7, hard, n);
    }
  }
  compare("hard info-first", hs, hf, hard);
  compare("soft queue+stamps", ks, kq1s, soft);
  compare("hard queue+stamps", hs, hq1s, hard);

  sustained(ks, soft, 300);   // clock warm-up
  stamp_run("soft_static", kss, soft, d_stamps, outdir);
  stamp_run("soft_queue_hop0", kq0s, soft, d_stamps, outdir);
  stamp_run("soft_queue_hop1", kq1s, soft, d_stamps, outdir);
  stamp_run("hard_static", hss, hard, d_stamps, outdir);
  stamp_run("hard_queue_hop0", hq0s, hard, d_stamps, outdir);
  stamp_run("hard_queue_hop1", hq1s, hard, d_stamps, outdir);

  // paired ABBA timing against the static walk, 40 launches per leg, 4 quadruples
  auto abba = [&](const char* name, Kern A, Kern B, const Setup& s) {
    sustained(A, s, 100);
    double r = 0, at = 0, bt = 0;
    for (int qd = 0; qd < 4; ++qd) {
      const float a0 = sustained(A, s, 40), b0 = sustained(B, s, 40), b1 = sustained(B, s, 40),
                  a1 = sustained(A, s, 40);
      r += (b0 + b1) / (a0 + a1);
      at += a0 + a1;
      bt += b0 + b1;
    }
    const double bits = (double)ng * 64 * blen;
    printf("%-34s static %.4f ms (%.1f Gbit/s)  variant %.4f ms (%.1f Gbit/s)  time ratio %.3f\n", name,
           at / 8, bits / (at / 8 * 1e-3) / 1e9, bt / 8, bits / (bt / 8 * 1e-3) / 1e9, r / 4);
  };
  soft.a.out = d_out_a;
  hard.a.out = d_out_a;
  abba("soft K=7 (headline): queue hop0", ks, kq0, soft);
  abba("soft K=7 (headline): queue hop1", ks, kq1, soft);
  abba("soft K=7 (headline): queue hop7", ks, kq7, soft);
  abba("hard K=7 (config 4): info-first", hs, hf, hard);
  abba("hard K=7 (config 4): queue hop0", hs, hq0, hard);
  abba("hard K=7 (config 4): queue hop1", hs, hq1, hard);
  abba("hard K=7 (config 4): queue hop7", hs, hq7, hard);

  // K = 9: 32 frames = 800,000 blocks of T = 48 (the bench's K = 9 batch)
  {
    constexpr CodeSpec kK9 = kMultiCodes[2], kK9T = kMultiCodes[3];
    const int nb9 = 800000, T9 = 48;
    void* d_slot;
    const size_t slot = std::max(wide_slot_bytes<kK9, 2>(40), multi2_slot_bytes<kK9T, 40>());
    CHECK(hipMalloc(&d_slot, slot * 8192));
    hipLaunchKernelGGL(fill_soft, dim3(8192), dim3(256), 0, 0, d_soft, (size_t)nb9 * T9 * 4);
    Setup k9{};
    k9.a = soft.a;
    k9.a.T = T9;
    k9.a.nblocks = nb9;
    k9.a.dec = d_slot;
    k9.a.out = d_out_a;
    const Kern ws = viterbi_wide_persist<kK9, 40, 0, 2>, wq = viterbi_wide_persist<kK9, 40, QU | H7, 2>;
    const Kern ms = viterbi_multi2_slot<kK9T, 40>, mq = viterbi_multi2_slot<kK9T, 40, 7, QU | H7>;
    auto cmp9 = [&](const char* name, Kern ref, Kern k, int bpg) {
      Setup s = k9;
      const int g = (nb9 + bpg - 1) / bpg;
      for (uint8_t* o : {d_out_a, d_out_b}) CHECK(hipMemset(o, 0xA5, (size_t)nb * 8));
      s.a.out = d_out_a;
      hipLaunchKernelGGL(ref, dim3(grid_of(ref, g)), dim3(64), 0, 0, s.a, g);
      s.a.out = d_out_b;
      for (int rep = 0; rep < 3; ++rep) hipLaunchKernelGGL(k, dim3(grid_of(k, g)), dim3(64), 0, 0, s.a, g);
      CHECK(hipDeviceSynchronize());
      std::vector<uint8_t> x((size_t)nb9 * 7), y((size_t)nb9 * 7);
      CHECK(hipMemcpy(x.data(), d_out_a, x.size(), hipMemcpyDeviceToHost));
      CHECK(hipMemcpy(y.data(), d_out_b, y.size(), hipMemcpyDeviceToHost));
      printf("%s (%d groups): outputs %s the static walk's\n", name, g, x == y ? "identical to" : "DIFFER from");
      bad += x != y;
    };
    cmp9("K=9 wide queue", ws, wq, 64);
    cmp9("K=9 two-lane queue", ms, mq, 32);
    auto abba9 = [&](const char* name, Kern A, Kern B, int bpg) {
      Setup s = k9;
      s.ngroups = (nb9 + bpg - 1) / bpg;
      sustained(A, s, 100);
      double r = 0, at = 0, bt = 0;
      for (int qd = 0; qd < 4; ++qd) {
        const float a0 = sustained(A, s, 20), b0 = sustained(B, s, 20), b1 = sustained(B, s, 20),
                    a1 = sustained(A, s, 20);
        r += (b0 + b1) / (a0 + a1);
        at += a0 + a1;
        bt += b0 + b1;
      }
      const double bits = (double)nb9 * 40;
      printf("%-34s static %.4f ms (%.1f Gbit/s)  variant %.4f ms (%.1f Gbit/s)  time ratio %.3f\n", name,
             at / 8, bits / (at / 8 * 1e-3) / 1e9, bt / 8, bits / (bt / 8 * 1e-3) / 1e9, r / 4);
    };
    abba9("K=9 wide (config 3): queue", ws, wq, 64);
    abba9("K=9 two-lane (textbook): queue", ms, mq, 32);
  }
  return bad ? 2 : 0;
}
