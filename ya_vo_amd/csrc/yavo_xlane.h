// yavo_xlane.h -- butterfly exchanges inside a wave64 without the LDS crossbar.
//
// __shfl_xor compiles to ds_bpermute_b32: an LDS-unit round trip (address VALU, the permute, an lgkmcnt wait) per
// dword.  A reduction tree of a few levels is that latency times its depth.  These helpers give the same lane
// pairing from the VALU side:
//   xor 1, 2   one DPP quad_perm mov per dword
//   xor 4      quad_perm(3,2,1,0) then row_half_mirror: lane l reads l^3, then l^7 of that, i.e. l^4
//   xor 8      row_ror:8 (a rotation by half a 16-lane row is its own inverse)
//   xor 16/32  gfx950's v_permlane16_swap / v_permlane32_swap, which exchange half-rows / half-waves of two
//              registers in place.
// Every DPP control used reads a lane of the same row, so the result never depends on bound_ctrl.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace yavo {
namespace xl {

template <int CTRL>
__device__ __forceinline__ uint32_t dpp(uint32_t v) {
    return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, CTRL, 0xf, 0xf, false);
}

// v of lane (l ^ OFF), OFF in {1, 2, 4, 8}
template <int OFF>
__device__ __forceinline__ uint32_t xor_row(uint32_t v) {
    static_assert(OFF == 1 || OFF == 2 || OFF == 4 || OFF == 8, "in-row butterflies only");
    if constexpr (OFF == 1) return dpp<0xB1>(v);                 // quad_perm(1,0,3,2)
    else if constexpr (OFF == 2) return dpp<0x4E>(v);            // quad_perm(2,3,0,1)
    else if constexpr (OFF == 4) return dpp<0x141>(dpp<0x1B>(v)); // row_half_mirror(quad_perm(3,2,1,0))
    else return dpp<0x128>(v);                                    // row_ror:8
}

template <int OFF>
__device__ __forceinline__ double xor_row_f64(double v) {
    const uint64_t b = __builtin_bit_cast(uint64_t, v);
    const uint32_t lo = xor_row<OFF>((uint32_t)b), hi = xor_row<OFF>((uint32_t)(b >> 32));
    return __builtin_bit_cast(double, ((uint64_t)hi << 32) | lo);
}

// v of lane L of this lane's 16-lane row (DPP row_newbcast, gfx90a+): a row-wide broadcast without the LDS unit
template <int L>
__device__ __forceinline__ double row_bcast_f64(double v) {
    static_assert(L >= 0 && L < 16, "a lane of the row");
    const uint64_t b = __builtin_bit_cast(uint64_t, v);
    const uint32_t lo = dpp<0x150 + L>((uint32_t)b), hi = dpp<0x150 + L>((uint32_t)(b >> 32));
    return __builtin_bit_cast(double, ((uint64_t)hi << 32) | lo);
}

template <int OFF>
__device__ __forceinline__ int xor_row_i32(int v) {
    return (int)xor_row<OFF>((uint32_t)v);
}

// Half-exchange of a reduce-scatter level with partner distance OFF in {16, 32}: the lane with bit OFF clear holds
// lo of its own and needs its partner's lo; the lane with bit OFF set holds hi and needs its partner's hi.  One
// permlane swap of (lo, hi) leaves, in every lane, its own kept value in one register and the partner's matching
// value in the other; the returned pair is {own-or-partner, partner-or-own} and their sum is the level's output.
template <int OFF>
__device__ __forceinline__ void swap_halves(uint32_t& lo, uint32_t& hi) {
    static_assert(OFF == 16 || OFF == 32, "permlane swaps exchange half-rows or half-waves");
    if constexpr (OFF == 32) {
        const auto r = __builtin_amdgcn_permlane32_swap(lo, hi, false, false);
        lo = r[0];
        hi = r[1];
    } else {
        const auto r = __builtin_amdgcn_permlane16_swap(lo, hi, false, false);
        lo = r[0];
        hi = r[1];
    }
}

template <int OFF>
__device__ __forceinline__ void swap_halves_f64(double& lo, double& hi) {
    const uint64_t a = __builtin_bit_cast(uint64_t, lo), b = __builtin_bit_cast(uint64_t, hi);
    uint32_t a0 = (uint32_t)a, a1 = (uint32_t)(a >> 32), b0 = (uint32_t)b, b1 = (uint32_t)(b >> 32);
    swap_halves<OFF>(a0, b0);
    swap_halves<OFF>(a1, b1);
    lo = __builtin_bit_cast(double, ((uint64_t)a1 << 32) | a0);
    hi = __builtin_bit_cast(double, ((uint64_t)b1 << 32) | b0);
}

}  // namespace xl
}  // namespace yavo
