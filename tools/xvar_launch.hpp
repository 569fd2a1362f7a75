// tools/xvar_launch.hpp -- per-type entry points of tools/xvar.py's timing
// variants (included by cuzfp_amd/csrc/kernels.hpp under CUZFP_XVAR; never
// part of the product library).  A variant instantiates the fast-gather
// kernels of one dimensionality (CUZFP_XVAR_DIMS, default 3) for its scalar
// type, and CUZFP_XVAR_STUB units none at all, so that a timing variant of
// the 3D f32 kernels compiles in a fraction of the product build's time.
#pragma once
#ifndef CUZFP_XVAR_DIMS
#define CUZFP_XVAR_DIMS 3
#endif
template <typename Scalar>
int launch_encode_type(const Problem& p, const void* data, bool fast, uint64_t* stream,
                       uint32_t wave0, uint32_t nwaves, hipStream_t st) {
#if !defined(CUZFP_XVAR_STUB)
  if (p.dims == CUZFP_XVAR_DIMS && fast)
    return launch_encode_t<Scalar, CUZFP_XVAR_DIMS>(data, p.g, fast, stream, wave0, nwaves, st);
#endif
  (void)p, (void)data, (void)fast, (void)stream, (void)wave0, (void)nwaves, (void)st;
  return CUZFP_ERROR_UNSUPPORTED_TYPE;
}
template <typename Scalar>
int launch_decode_type(const Problem& p, const uint64_t* stream, bool fast, void* data,
                       uint32_t wave0, uint32_t nwaves, hipStream_t st) {
#if !defined(CUZFP_XVAR_STUB)
  if (p.dims == CUZFP_XVAR_DIMS && fast)
    return launch_decode_t<Scalar, CUZFP_XVAR_DIMS>(stream, p.g, fast, data, wave0, nwaves, st);
#endif
  (void)p, (void)data, (void)fast, (void)stream, (void)wave0, (void)nwaves, (void)st;
  return CUZFP_ERROR_UNSUPPORTED_TYPE;
}
