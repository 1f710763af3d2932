// LDS reads, waits and barriers as inline asm, for kernels that keep LDS-DMA loads
// (global_load_lds / buffer_load ... lds) in flight across their LDS reads: hipcc cannot
// tell the ring slot being read from the slots still being filled, so it drains vmcnt(0)
// before every plain LDS read, which would wait for every tile in flight.  The caller waits
// lgkmcnt itself (asm_wait_lgkm) and then marks the values landed (asm_landed), so nothing
// the compiler schedules can consume them before the wait.
#pragma once
#include "common.h"

namespace osw {

typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
typedef unsigned u32x2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ unsigned lds_addr(const h16* p) { return (unsigned)(uintptr_t)(OSW_LDS const h16*)p; }
__device__ __forceinline__ h16x8 asm_read_b128(const h16* p) {
    u32x4 v;
    asm volatile("ds_read_b128 %0, %1" : "=v"(v) : "v"(lds_addr(p)) : "memory");
    return __builtin_bit_cast(h16x8, v);
}
// ds_read_b64_tr_b16: per 16-lane group, lane 4q + p addresses row q, columns 4p .. 4p+3 of a
// 4 x 16 block; lane i receives column i of the 4 rows
__device__ __forceinline__ h16x4 asm_read_tr(const h16* p) {
    u32x2 v;
    asm volatile("ds_read_b64_tr_b16 %0, %1" : "=v"(v) : "v"(lds_addr(p)) : "memory");
    return __builtin_bit_cast(h16x4, v);
}
__device__ __forceinline__ float asm_read_f32(const float* p) {
    float v;
    asm volatile("ds_read_b32 %0, %1" : "=v"(v) : "v"((unsigned)(uintptr_t)(OSW_LDS const float*)p) : "memory");
    return v;
}
__device__ __forceinline__ void asm_wait_lgkm() { asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory"); }
template <class T>
__device__ __forceinline__ void asm_landed(T& v) { asm volatile("" : "+v"(v)); }

template <int N>
__device__ __forceinline__ void asm_wait_vmcnt() {
    static_assert(N >= 0 && N < 64, "vmcnt range");
    asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

// LDS writes of every wave visible, the wave's outstanding global loads untouched
__device__ __forceinline__ void asm_lds_barrier() {
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
}

}  // namespace osw
