// tick_latency.cpp — dev tool: wall time of ONE host-memory engine call per
// batch, the way a TUN / socket event loop calls it each tick
// (util/tuntap/tuntap_adapter.cpp:5-21 inside
// util/tcp_minnow_socket/tcp_minnow_socket.h:138-164: a few datagrams per
// tick, results needed before the next).  Loads one or more builds of
// libicsum.so side by side (dlopen, RTLD_LOCAL) and times them interleaved on
// the same buffers; every build's outputs must equal the first's.
//   g++ -O2 -std=c++17 -I../../include tick_latency.cpp -o tick_latency -ldl
//   tick_latency libA.so[@FORCE] [libB.so[@FORCE] ...]
// (@FORCE: that context is created with ICSUM_FORCE=FORCE, e.g.
// lib.so@tick_inline=0 — one build, two dispatch choices, one process)
// Environment: TICK_OPS (comma list of verify, verify_off, checksum, checksum_off, wrap;
// default all), TICK_SIZES (comma list of batch sizes, default 1..8192),
// TICK_MEM (pinned | pageable, default both), TICK_CALLS (timed calls per
// round, default 200), TICK_GAP_US (host busy time before each call, outside
// the timed call: a loop that does other work between ticks; default 0).
// Checksum calls pass per-segment inits (the NS
// workload's pseudo-header sums).  bench.py's host_inclusive runs it as
// TICK_OPS=checksum TICK_SIZES=1,16 TICK_MEM=pinned (built by build()).
#include <dlfcn.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <chrono>
#include <random>
#include <string>
#include <vector>

#include "icsum.h"

namespace {

struct Lib {
  std::string path;
  ics_ctx* ctx = nullptr;
  int (*create)(int, ics_ctx**);
  int (*destroy)(ics_ctx*);
  int (*host_alloc)(ics_ctx*, void**, size_t);
  int (*checksum_host)(ics_ctx*, const void*, const uint64_t*, uint64_t, uint64_t, const uint32_t*, uint16_t*,
                       uint64_t);
  int (*ipv4_host)(ics_ctx*, void*, const uint64_t*, uint64_t, uint64_t, uint64_t, int, uint16_t*, uint16_t*,
                   uint8_t*);
  int (*wrap_host)(ics_ctx*, void*, const uint64_t*, uint64_t, uint64_t, uint64_t, const ics_tcp_msg*);
  const char* (*last_error)();
};

template <typename F>
void sym(void* h, const char* name, F& f) {
  f = reinterpret_cast<F>(dlsym(h, name));
  if (!f) {
    fprintf(stderr, "missing %s\n", name);
    exit(1);
  }
}

Lib open_lib(const char* arg) {
  Lib l;
  l.path = arg;
  const std::string a(arg);
  const size_t at = a.find('@');
  const std::string path = a.substr(0, at);
  void* h = dlopen(path.c_str(), RTLD_NOW | RTLD_LOCAL);
  if (!h) {
    fprintf(stderr, "dlopen %s: %s\n", path.c_str(), dlerror());
    exit(1);
  }
  sym(h, "ics_create", l.create);
  sym(h, "ics_destroy", l.destroy);
  sym(h, "ics_host_alloc", l.host_alloc);
  sym(h, "ics_checksum_batch_host", l.checksum_host);
  sym(h, "ics_ipv4_tcp_batch_host", l.ipv4_host);
  sym(h, "ics_tcp_wrap_batch_host", l.wrap_host);
  sym(h, "ics_last_error", l.last_error);
  if (at != std::string::npos) setenv("ICSUM_FORCE", a.substr(at + 1).c_str(), 1);
  const int rc = l.create(0, &l.ctx);
  unsetenv("ICSUM_FORCE");
  if (rc != ICS_OK) {
    fprintf(stderr, "ics_create: %s\n", l.last_error());
    exit(1);
  }
  return l;
}

void check(const Lib& l, int rc) {
  if (rc != ICS_OK) {
    fprintf(stderr, "%s: %s\n", l.path.c_str(), l.last_error());
    exit(1);
  }
}

using clk = std::chrono::steady_clock;

double pct(std::vector<double> v, double p) {
  std::sort(v.begin(), v.end());
  return v[size_t(p * double(v.size() - 1))];
}

}  // namespace

int main(int argc, char** argv) {
  if (argc < 2) {
    fprintf(stderr, "usage: %s lib.so [lib.so ...]\n", argv[0]);
    return 2;
  }
  std::vector<Lib> libs;
  for (int i = 1; i < argc; ++i) libs.push_back(open_lib(argv[i]));
  constexpr uint64_t kL = 1500, kMaxN = 8192;
  std::vector<uint8_t> pageable(kMaxN * kL);
  std::mt19937_64 rng(7);
  for (auto& b : pageable) b = uint8_t(rng());
  uint8_t* pinned = nullptr;
  check(libs[0], libs[0].host_alloc(libs[0].ctx, reinterpret_cast<void**>(&pinned), kMaxN * kL));
  memcpy(pinned, pageable.data(), kMaxN * kL);
  std::vector<ics_tcp_msg> msgs(kMaxN);
  for (uint64_t i = 0; i < kMaxN; ++i) {
    msgs[i] = ics_tcp_msg{0x0a000001u, 0x0a000002u, uint32_t(rng()), uint32_t(rng()), 40000, 80, 64000, 0x10, 128,
                          0, 0};
  }
  std::vector<uint64_t> sizes = {1, 4, 16, 64, 256, 512, 1024, 4096, 8192};
  if (const char* e = getenv("TICK_SIZES")) {
    sizes.clear();
    for (const char* p = e; *p;) {
      char* end = nullptr;
      const unsigned long long v = strtoull(p, &end, 10);
      if (end == p || v == 0 || v > kMaxN) {
        fprintf(stderr, "TICK_SIZES: sizes 1..%llu, comma-separated\n", (unsigned long long)kMaxN);
        return 2;
      }
      sizes.push_back(v);
      p = *end == ',' ? end + 1 : end;
    }
  }
  const char* mem_only = getenv("TICK_MEM");
  std::vector<uint32_t> inits(kMaxN);
  for (auto& v : inits) v = uint32_t(rng());
  const char* ops[] = {"verify", "verify_off", "checksum", "checksum_off", "wrap"};
  const char* only = getenv("TICK_OPS");  // comma list of ops to run (default: all)
  std::vector<uint64_t> offs(kMaxN + 1);
  for (uint64_t i = 0; i <= kMaxN; ++i) offs[i] = i * kL;
  const int rounds = 5, calls = getenv("TICK_CALLS") ? std::max(10, atoi(getenv("TICK_CALLS"))) : 200;
  const double gap_us = getenv("TICK_GAP_US") ? atof(getenv("TICK_GAP_US")) : 0.0;
  // every (build, op) pair of a size and memory kind is timed interleaved call
  // by call, the first pair rotating per call: each pair's calls follow every
  // other pair's equally often (blocks of calls per build or per op measured
  // ~1 us position biases on identical code)
  struct Var {
    size_t k;
    const char* op;
  };
  for (int mem = 0; mem < 2; ++mem) {
    if (mem_only && strcmp(mem_only, mem ? "pinned" : "pageable")) continue;
    for (uint64_t n : sizes) {
      uint8_t* src = mem ? pinned : pageable.data();
      std::vector<Var> vars;
      for (const char* op : ops)
        if (!only || strstr(only, op))
          for (size_t k = 0; k < libs.size(); ++k) vars.push_back({k, op});
      if (only) {  // exact names only ("verify" must not select "verify_off")
        std::vector<Var> keep;
        for (const Var& v : vars) {
          const size_t len = strlen(v.op);
          for (const char* p = strstr(only, v.op); p; p = strstr(p + 1, v.op))
            if ((p == only || p[-1] == ',') && (p[len] == ',' || p[len] == 0)) {
              keep.push_back(v);
              break;
            }
        }
        vars.swap(keep);
      }
      std::vector<std::vector<double>> t(vars.size());
      std::vector<std::vector<uint8_t>> res(vars.size(), std::vector<uint8_t>(n * kL + n * 5));
      for (int r = 0; r < rounds; ++r)
        for (int c = 0; c < calls + 10; ++c)
          for (size_t jj = 0; jj < vars.size(); ++jj) {
            const size_t j = (jj + size_t(c)) % vars.size();
            const Lib& l = libs[vars[j].k];
            const char* op = vars[j].op;
            uint16_t* a = reinterpret_cast<uint16_t*>(res[j].data());
            uint16_t* b = a + n;
            uint8_t* st = reinterpret_cast<uint8_t*>(b + n);
            if (gap_us > 0)
              for (const auto g0 = clk::now(); std::chrono::duration<double, std::micro>(clk::now() - g0).count() < gap_us;) {
              }
            const auto t0 = clk::now();
            if (!strcmp(op, "verify_off"))
              check(l, l.ipv4_host(l.ctx, src, offs.data(), 0, 0, n, ICS_MODE_VERIFY, a, b, st));
            else if (op[0] == 'v')
              check(l, l.ipv4_host(l.ctx, src, nullptr, kL, kL, n, ICS_MODE_VERIFY, a, b, st));
            else if (!strcmp(op, "checksum_off"))
              check(l, l.checksum_host(l.ctx, src, offs.data(), 0, 0, inits.data(), a, n));
            else if (op[0] == 'c')
              check(l, l.checksum_host(l.ctx, src, nullptr, kL, kL, inits.data(), a, n));
            else
              check(l, l.wrap_host(l.ctx, src, nullptr, kL, kL, n, msgs.data()));
            if (c >= 10) t[j].push_back(std::chrono::duration<double, std::micro>(clk::now() - t0).count());
            if (op[0] == 'w') memcpy(res[j].data() + n * 5, src, n * kL);  // the wrapped wire bytes
          }
      for (size_t j = 0; j < vars.size(); ++j) {
        size_t first = j;  // the same op's first build
        while (first > 0 && !strcmp(vars[first - 1].op, vars[j].op)) --first;
        const bool same = res[j] == res[first];
        printf("{\"op\": \"%s\", \"mem\": \"%s\", \"n\": %llu, \"bytes\": %llu, \"lib\": \"%s\", \"p10_us\": %.2f, "
               "\"p50_us\": %.2f, \"p90_us\": %.2f, \"gap_us\": %.1f, \"same_as_first\": %s}\n",
               vars[j].op, mem ? "pinned" : "pageable", (unsigned long long)n, (unsigned long long)(n * kL),
               libs[vars[j].k].path.c_str(), pct(t[j], 0.1), pct(t[j], 0.5), pct(t[j], 0.9), gap_us,
               same ? "true" : "false");
        fflush(stdout);
      }
    }
  }
  for (auto& l : libs) l.destroy(l.ctx);
  return 0;
}
