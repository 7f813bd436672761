// Microbenchmark: the XCD-hierarchical grid barrier (MI355X_MICROARCH.md "barrier-xcd") in a
// persistent kernel, per barrier, at a given grid -- the form VERDICT r04 item 2 asked to
// re-measure before a persistent C5 drain kernel.  Diagnostic only.
//   arrive: __syncthreads; lane 0: release fence (agent), relaxed add to its XCC's counter
//   (HW_REG_XCC_ID); the XCC's last arriver adds to the top counter; the last top arriver
//   bumps the generation (relaxed agent store); every other lane 0 polls the generation with
//   relaxed sc1 loads + s_sleep; then ONE acquire fence (agent), vmcnt(0), __syncthreads.
//   Per-XCC group sizes come from a census at kernel start (one flat counter pass).
//   Every spin is bounded: a timeout sets *err and the wave leaves.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e_), __LINE__); exit(1); } } while (0)

typedef __attribute__((address_space(1))) unsigned int gu32;
constexpr int kLine = 32;  // words per 128-B line
struct Bar {
  unsigned int census[8 * kLine];  // WGs per XCC (line each)
  unsigned int cnt[8 * kLine];     // arrivals per XCC
  unsigned int top[kLine];
  unsigned int gen[kLine];
  unsigned int start[kLine];
};

__device__ __forceinline__ unsigned int xcc_id() {
  unsigned int v;
  asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(v));
  return v & 7u;
}
__device__ __forceinline__ unsigned int ld_rlx(unsigned int* p) {
  return __hip_atomic_load((gu32*)p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ unsigned int add_rlx(unsigned int* p, unsigned int v) {
  return __hip_atomic_fetch_add((gu32*)p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// returns false on timeout
__device__ bool barrier_xcd(Bar* b, unsigned int xcc, unsigned int nxcc_wg, unsigned int ngroups, unsigned int& gen,
                            int* err) {
  __syncthreads();
  __shared__ int s_ok;
  if (threadIdx.x == 0) {
    s_ok = 1;
    const unsigned int g = gen;
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    bool last = false;
    if (add_rlx(&b->cnt[xcc * kLine], 1u) == (g + 1) * nxcc_wg - 1) {  // monotonic per-XCC count
      if (add_rlx(&b->top[0], 1u) == (g + 1) * ngroups - 1) {
        __hip_atomic_store((gu32*)&b->gen[0], g + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        last = true;
      }
    }
    if (!last) {
      long spins = 0;
      while (ld_rlx(&b->gen[0]) == g) {
        __builtin_amdgcn_s_sleep(1);
        if (++spins > 4000000) { *err = 1; s_ok = 0; break; }
      }
    }
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
  gen++;
  __syncthreads();
  return s_ok != 0;
}

__global__ void __launch_bounds__(256) k_persist(Bar* b, int iters, int* err, unsigned int* data, unsigned int nblocks,
                                                 unsigned long long* cycles) {
  __shared__ unsigned int s_n, s_groups;
  const unsigned int xcc = xcc_id();
  if (threadIdx.x == 0) {
    add_rlx(&b->census[xcc * kLine], 1u);
    // census barrier: everyone arrived once on a flat counter
    add_rlx(&b->start[0], 1u);
    long spins = 0;
    while (ld_rlx(&b->start[0]) < nblocks) {
      __builtin_amdgcn_s_sleep(1);
      if (++spins > 4000000) { *err = 2; break; }
    }
    unsigned int groups = 0;
    for (int k = 0; k < 8; ++k) groups += ld_rlx(&b->census[k * kLine]) ? 1u : 0u;
    s_n = ld_rlx(&b->census[xcc * kLine]);
    s_groups = groups;
  }
  __syncthreads();
  if (*(volatile int*)err) return;
  unsigned int gen = 0;
  const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
  for (int i = 0; i < iters; ++i) {
    data[blockIdx.x * 256 + threadIdx.x] += 1;  // a little work per phase
    if (!barrier_xcd(b, xcc, s_n, s_groups, gen, err)) return;
  }
  const unsigned long long t1 = __builtin_amdgcn_s_memrealtime();
  if (threadIdx.x == 0 && blockIdx.x == 0) cycles[0] = t1 - t0;  // 100 MHz ticks
}

int main(int argc, char** argv) {
  const int iters = argc > 1 ? atoi(argv[1]) : 20000;
  Bar* b; int* err; unsigned int* data; unsigned long long* cyc;
  CK(hipMalloc(&b, sizeof(Bar)));
  CK(hipMalloc(&err, 4));
  CK(hipMalloc(&data, 2048 * 256 * 4)); CK(hipMemset(data, 0, 2048 * 256 * 4));
  CK(hipMalloc(&cyc, 8));
  hipDeviceProp_t prop; CK(hipGetDeviceProperties(&prop, 0));
  int nb_per_cu = 0;
  CK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb_per_cu, k_persist, 256, 0));
  printf("CUs %d, resident blocks per CU (query) %d\n", prop.multiProcessorCount, nb_per_cu);
  const int grids[] = {256, 391, 512};
  for (int gi = 0; gi < 3; ++gi) {
    const unsigned int nb = grids[gi];
    if ((int)nb > prop.multiProcessorCount * 2) continue;  // at most 2 blocks per CU: resident
    for (int rep = 0; rep < 2; ++rep) {
      CK(hipMemset(b, 0, sizeof(Bar)));
      CK(hipMemset(err, 0, 4));
      int n = iters;
      hipLaunchKernelGGL(k_persist, dim3(nb), dim3(256), 0, 0, b, n, err, data, nb, cyc);
      CK(hipDeviceSynchronize());
      int e = 0; unsigned long long c = 0;
      CK(hipMemcpy(&e, err, 4, hipMemcpyDeviceToHost));
      CK(hipMemcpy(&c, cyc, 8, hipMemcpyDeviceToHost));
      printf("barrier-xcd grid %u: %s %.3f us per barrier (%d barriers)\n", nb, e ? "TIMEOUT" : "ok",
             c * 0.01 / n, n);
      if (e) return 1;
    }
  }
  return 0;
}
