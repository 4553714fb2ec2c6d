// ol_dsp_amd/csrc/lds_flags.h -- progress counters in LDS for the role-pipelined kernels (the fused
// chain, the Svf voice): a producer wave publishes "chunks done" with a workgroup-scope release
// store, a consumer waits with acquire loads until the chunk it needs is published (or the buffer
// it will overwrite is released).  Counters only grow.  Unlike a workgroup barrier per step, a
// wave waits only for the waves it exchanges data with, so a role may run ahead by the depth of
// its queue and the pipeline runs at the speed of its slowest role instead of the slowest role of
// every step.  Release/acquire at workgroup scope order LDS accesses only (s_waitcnt lgkmcnt):
// prefetched global loads stay in flight across them.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace olfx {

__device__ __forceinline__ uint32_t flag_get(const uint32_t *f) {
    return __hip_atomic_load(f, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP);
}
__device__ __forceinline__ void flag_put(uint32_t *f, uint32_t v) {
    __hip_atomic_store(f, v, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
}
// spin (with s_sleep) until cond(); every wait targets a counter that another role advances
// without first waiting on the waiting role, so the pipeline cannot deadlock
template <class Cond>
__device__ __forceinline__ void wait_for(Cond &&cond) {
    while (!cond()) __builtin_amdgcn_s_sleep(1);
}

}  // namespace olfx
