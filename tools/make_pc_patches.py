#!/usr/bin/env python3
"""Regenerates the diagnostic patches of pyramid_pc.hip from the current
source (tools/patches/pc_ablation.patch: timing ablations, -DPC_ABL=<bits>;
tools/patches/pc_stamps.patch: per-wave wait stamps read by
tools/pc_stamps.py).  Built with tools/build_patch.sh.
    python3 tools/make_pc_patches.py"""
import difflib
import os

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = os.path.join(ROOT, "sift-gpu_amd", "csrc", "pyramid_pc.hip")


def rep(s, a, b, cnt=1):
    assert s.count(a) == cnt, (a, s.count(a))
    return s.replace(a, b)


def ablation(s):
    s = rep(s, '''constexpr int kPollMax = 1 << 20;''', '''// Timing ablations (garbage results): PC_ABL & 1 = no plane stores, & 2 = no
// LDS-DMA loads, & 16 = no FMAs in the consumers' row and column passes, & 32 =
// no base-blur arithmetic in the producer
#ifndef PC_ABL
#define PC_ABL 0
#endif
constexpr int kPollMax = 1 << 20;''')
    s = rep(s, '''__device__ __forceinline__ void pc_store4(PRsrc rs, unsigned voff, float4 v) {
''', '''__device__ __forceinline__ void pc_store4(PRsrc rs, unsigned voff, float4 v) {
  if constexpr (PC_ABL & 1) return;
''')
    s = rep(s, '''__device__ __forceinline__ void pc_store2(PRsrc rs, unsigned voff, float a, float b) {
''', '''__device__ __forceinline__ void pc_store2(PRsrc rs, unsigned voff, float a, float b) {
  if constexpr (PC_ABL & 1) return;
''')
    s = rep(s, '''__device__ __forceinline__ void pc_dma(unsigned lds_byte, unsigned voff, PRsrc rs, unsigned soff) {
''', '''__device__ __forceinline__ void pc_dma(unsigned lds_byte, unsigned voff, PRsrc rs, unsigned soff) {
  if constexpr (PC_ABL & 2) return;
''')
    s = rep(s, '''__device__ __forceinline__ void pc_scatter(float (&acc)[P], float h, std::integer_sequence<int, I...>) {
''', '''__device__ __forceinline__ void pc_scatter(float (&acc)[P], float h, std::integer_sequence<int, I...>) {
  if constexpr (PC_ABL & 16) {
    acc[((R - W) % P + P) % P] = h;
    return;
  }
''')
    s = rep(s, '''  for (int k = 1; k <= W1; ++k) {
    float pk[4];''', '''  for (int k = 1; k <= ((PC_ABL & 16) ? 0 : W1); ++k) {
    float pk[4];''')
    s = rep(s, '''      for (int k = 1; k <= 4; ++k) {
        float pk[4];''', '''      for (int k = 1; k <= ((PC_ABL & 32) ? 0 : 4); ++k) {
        float pk[4];''')
    s = rep(s, '''      for (int k = 1; k <= 4; ++k) {
        float pk[kPB];''', '''      for (int k = 1; k <= ((PC_ABL & 32) ? 0 : 4); ++k) {
        float pk[kPB];''')
    return s


def stamps(s):
    s = rep(s, '''#include "../build/sym_coefs.inc"
''', '''#include "../build/sym_coefs.inc"

// ---- stamps (diagnostic build only: tools/build_patch.sh pcstamps
// tools/patches/pc_stamps.patch; read by tools/pc_stamps.py) ----
// Per (octave, block, wave): [0] cycles in the wave, [1] cycles spent in
// pc_wait_ge / pc_wait_done, [2] waits that polled at least once, [3] steps.
constexpr int kPsBlocks = 16384;
__device__ unsigned long long g_pc_stamps[5][kPsBlocks][4][4];
struct PsAcc {
  unsigned long long wait = 0, nwait = 0;
};
__device__ __forceinline__ void ps_flush(int oct, int wave, const PsAcc& ps, unsigned long long t0, int steps) {
  const int lane = threadIdx.x & 63;
  if (lane < 4 && blockIdx.x < kPsBlocks) {
    const unsigned long long v = lane == 0 ? __builtin_amdgcn_s_memtime() - t0 : lane == 1 ? ps.wait
                                 : lane == 2 ? ps.nwait : (unsigned long long)steps;
    unsigned long long* slot = &g_pc_stamps[oct < 5 ? oct : 4][blockIdx.x][wave][lane];
    *slot = *slot + v;
  }
}
''')
    s = rep(s, '''__device__ __forceinline__ void pc_wait_ge(const int* w, int v, int* err) {
  int it = 0;''', '''__device__ __forceinline__ void pc_wait_ge(const int* w, int v, int* err, PsAcc& ps) {
  const unsigned long long t0 = __builtin_amdgcn_s_memtime();
  if (pc_peek(w) < v) ps.nwait += 1;
  int it = 0;''')
    s = rep(s, '''__device__ __forceinline__ void pc_wait_done(const PcFlags& f, int v, int* err) {
  int it = 0;''', '''__device__ __forceinline__ void pc_wait_done(const PcFlags& f, int v, int* err, PsAcc& ps) {
  const unsigned long long t0 = __builtin_amdgcn_s_memtime();
  if (min(min(pc_peek(&f.done[0]), pc_peek(&f.done[1])), pc_peek(&f.done[2])) < v) ps.nwait += 1;
  int it = 0;''')
    s = rep(s, '''    __builtin_amdgcn_s_sleep(1);
  }
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
}''', '''    __builtin_amdgcn_s_sleep(1);
  }
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  ps.wait += __builtin_amdgcn_s_memtime() - t0;
}''', 2)
    s = rep(s, '''  int* err;                // sticky error word err[3] (kErrStall: a bounded wait expired)
};''', '''  int* err;                // sticky error word err[3] (kErrStall: a bounded wait expired)
  int oct;
};''')
    for fn in ("pc_producer0(const PcArgs& A, PcLds0& L", "pc_producerN(const PcArgs& A, PcLdsN& L"):
        s = rep(s, f'''__device__ __forceinline__ void {fn}, int b, int x0, int y0, int y1) {{
  const int lane = threadIdx.x & 63;''', f'''__device__ __forceinline__ void {fn}, int b, int x0, int y0, int y1) {{
  PsAcc ps;
  const unsigned long long ps_t0 = __builtin_amdgcn_s_memtime();
  const int lane = threadIdx.x & 63;''')
    s = rep(s, '''pc_wait_done(L.f, s - kPD + 1, A.err);''', '''pc_wait_done(L.f, s - kPD + 1, A.err, ps);''')
    s = rep(s, '''pc_wait_done(L.f, s + 2 - kPD + 1, A.err);''', '''pc_wait_done(L.f, s + 2 - kPD + 1, A.err, ps);''')
    s = rep(s, '''    pc_wave_sync();  // tr0 reads before the next step's writes (program order)
  }
}''', '''    pc_wave_sync();  // tr0 reads before the next step's writes (program order)
  }
  PC_WAIT_VM(0);
  ps_flush(A.oct, 0, ps, ps_t0, nsteps);
}''')
    s = rep(s, '''      issue(s + 2);
    }
  }
}''', '''      issue(s + 2);
    }
  }
  PC_WAIT_VM(0);
  ps_flush(A.oct, 0, ps, ps_t0, nsteps);
}''')
    s = rep(s, '''  using R_ = PcRole<C>;
''', '''  using R_ = PcRole<C>;
  PsAcc ps;
  const unsigned long long ps_t0 = __builtin_amdgcn_s_memtime();
''')
    s = rep(s, '''      pc_wait_ge(&L.f.pub, s + 1, A.err);''', '''      pc_wait_ge(&L.f.pub, s + 1, A.err, ps);''')
    s = rep(s, '''        pc_wait_ge(&L.f.hpub, s + 1, A.err);''', '''        pc_wait_ge(&L.f.hpub, s + 1, A.err, ps);''')
    s = rep(s, '''      pc_wait_ge(&L.f.hdone, s - kPH18 + 1, A.err);''', '''      pc_wait_ge(&L.f.hdone, s - kPH18 + 1, A.err, ps);''')
    s = rep(s, '''  if constexpr (!OCT0 && C == 0) pc_publish(&L.f.hdone, 1 << 30);
}''', '''  if constexpr (!OCT0 && C == 0) pc_publish(&L.f.hdone, 1 << 30);
  ps_flush(A.oct, C + 1, ps, ps_t0, nsteps);
}''')
    s = rep(s, '''  A.err = err;
  if (o == 0) {''', '''  A.err = err;
  A.oct = o;
  if (o == 0) {''')
    s += '''
extern "C" int sift_dbg_pc_stamps(unsigned long long* out, int reset) {
  if (out && hipMemcpyFromSymbol(out, HIP_SYMBOL(sift::g_pc_stamps), sizeof(sift::g_pc_stamps)) != hipSuccess)
    return -1;
  if (reset) {
    void* p = nullptr;
    if (hipGetSymbolAddress(&p, HIP_SYMBOL(sift::g_pc_stamps)) != hipSuccess ||
        hipMemset(p, 0, sizeof(sift::g_pc_stamps)) != hipSuccess || hipDeviceSynchronize() != hipSuccess)
      return -1;
  }
  return (int)sizeof(sift::g_pc_stamps);
}
'''
    return s


def write(name, new, old):
    d = difflib.unified_diff(old.splitlines(True), new.splitlines(True), "a/sift-gpu_amd/csrc/pyramid_pc.hip",
                             "b/sift-gpu_amd/csrc/pyramid_pc.hip")
    with open(os.path.join(ROOT, "tools", "patches", name), "w") as f:
        f.writelines(d)


def main():
    old = open(SRC).read()
    write("pc_ablation.patch", ablation(old), old)
    write("pc_stamps.patch", stamps(old), old)


if __name__ == "__main__":
    main()
