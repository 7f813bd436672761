// Microbenchmark: cost of a device-wide barrier in a persistent (cooperative) kernel vs a
// chain of dependent kernel launches, on one MI355X.  Diagnostic only.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e_), __LINE__); exit(1); } } while (0)

struct Bar { unsigned int count; unsigned int gen; unsigned int sub[8 * 32]; };

// flat: one counter; the last arriver bumps the generation.  Bounded spin: a block that
// waits too long sets *err and leaves (every wave exits).
__device__ bool grid_sync_flat(Bar* b, unsigned int nblocks, unsigned int& gen, int* err) {
  __syncthreads();
  if (threadIdx.x == 0) {
    const unsigned int g = gen;
    if (__hip_atomic_fetch_add(&b->count, 1u, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT) == nblocks - 1) {
      __hip_atomic_store(&b->count, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store(&b->gen, g + 1, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
    } else {
      long spins = 0;
      while (__hip_atomic_load(&b->gen, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT) == g) {
        __builtin_amdgcn_s_sleep(1);
        if (++spins > 20000000) { *err = 1; break; }
      }
    }
  }
  gen++;
  __syncthreads();
  return true;
}

// two-level: blocks arrive at sub-counter (blockIdx % 8) (the XCD of round-robin dispatch);
// the last of a group arrives at the top counter.
__device__ bool grid_sync_2l(Bar* b, unsigned int nblocks, unsigned int& gen, int* err) {
  __syncthreads();
  if (threadIdx.x == 0) {
    const unsigned int g = gen;
    const unsigned int grp = blockIdx.x & 7;
    const unsigned int gsz = nblocks / 8 + (grp < nblocks % 8 ? 1 : 0);
    unsigned int* sc = &b->sub[grp * 32];
    bool last = false;
    if (__hip_atomic_fetch_add(sc, 1u, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT) == gsz - 1) {
      __hip_atomic_store(sc, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (__hip_atomic_fetch_add(&b->count, 1u, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT) == 7) {
        __hip_atomic_store(&b->count, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_store(&b->gen, g + 1, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
        last = true;
      }
    }
    if (!last) {
      long spins = 0;
      while (__hip_atomic_load(&b->gen, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT) == g) {
        __builtin_amdgcn_s_sleep(1);
        if (++spins > 20000000) { *err = 1; break; }
      }
    }
  }
  gen++;
  __syncthreads();
  return true;
}

template <int MODE>
__global__ void __launch_bounds__(256) k_persist(Bar* b, int iters, int* err, unsigned int* data) {
  unsigned int gen = 0;
  for (int i = 0; i < iters; ++i) {
    if (*(volatile int*)err) break;
    // a little work: every thread touches one word
    data[blockIdx.x * 256 + threadIdx.x] += 1;
    if (MODE == 0) grid_sync_flat(b, gridDim.x, gen, err);
    else grid_sync_2l(b, gridDim.x, gen, err);
  }
}

__global__ void __launch_bounds__(256) k_step(unsigned int* data) { data[blockIdx.x * 256 + threadIdx.x] += 1; }

int main(int argc, char** argv) {
  const int nblocks = argc > 1 ? atoi(argv[1]) : 391;
  const int iters = argc > 2 ? atoi(argv[2]) : 20000;
  Bar* b; int* err; unsigned int* data;
  CK(hipMalloc(&b, sizeof(Bar))); CK(hipMemset(b, 0, sizeof(Bar)));
  CK(hipMalloc(&err, 4)); CK(hipMemset(err, 0, 4));
  CK(hipMalloc(&data, (size_t)nblocks * 256 * 4)); CK(hipMemset(data, 0, (size_t)nblocks * 256 * 4));
  hipEvent_t e0, e1; CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
  int nb_per_cu = 0;
  CK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb_per_cu, k_persist<0>, 256, 0));
  hipDeviceProp_t prop; CK(hipGetDeviceProperties(&prop, 0));
  printf("CUs %d, resident blocks per CU %d, grid %d\n", prop.multiProcessorCount, nb_per_cu, nblocks);
  if (nb_per_cu * prop.multiProcessorCount < nblocks) { printf("grid does not fit\n"); return 1; }
  for (int mode = 0; mode < 2; ++mode) {
    for (int rep = 0; rep < 2; ++rep) {
      int n = iters;
      void* args[] = {&b, &n, &err, &data};
      CK(hipMemset(b, 0, sizeof(Bar)));
      CK(hipEventRecord(e0));
      if (mode == 0) CK(hipLaunchCooperativeKernel((void*)k_persist<0>, dim3(nblocks), dim3(256), args, 0, 0));
      else CK(hipLaunchCooperativeKernel((void*)k_persist<1>, dim3(nblocks), dim3(256), args, 0, 0));
      CK(hipEventRecord(e1));
      CK(hipEventSynchronize(e1));
      float ms; CK(hipEventElapsedTime(&ms, e0, e1));
      int herr = 0; CK(hipMemcpy(&herr, err, 4, hipMemcpyDeviceToHost));
      printf("%s barrier: %.3f us per barrier (err %d)\n", mode == 0 ? "flat" : "two-level", 1000.0 * ms / iters, herr);
      if (herr) return 2;
    }
  }
  for (int rep = 0; rep < 2; ++rep) {
    CK(hipEventRecord(e0));
    for (int i = 0; i < iters; ++i) k_step<<<nblocks, 256>>>(data);
    CK(hipEventRecord(e1));
    CK(hipEventSynchronize(e1));
    float ms; CK(hipEventElapsedTime(&ms, e0, e1));
    printf("kernel chain: %.3f us per launch\n", 1000.0 * ms / iters);
  }
  return 0;
}
