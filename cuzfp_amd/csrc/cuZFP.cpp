// cuzfp_amd/csrc/cuZFP.cpp -- the reference's C++ surface (include/cuZFP.h) on
// top of the C-ABI (include/cuzfp_hip.h).
//
// Mirrors mclarsen/cuZFP src/cuZFP/cuZFP.cu:174-269:
//   compress   = setup_device_field + setup_device_stream (cuZFP.cu:107-155)
//                -> internal::encode<T> -> copy the stream back -> free
//   decompress = the same in reverse.
// Staging differs only where the reference wastes work: the stream is copied
// to the device only for decompress (cuZFP.cu:118-120 uploads the whole
// maximum-size buffer for compress too), only the bytes actually produced are
// copied back, and a contiguous output array is not uploaded before decoding
// (cuZFP.cu:221).  When both buffers are in host memory the pinned, chunked
// pipeline of cuzfp_hip_compress_host / cuzfp_hip_decompress_host is used.
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>

#include "../../include/cuZFP.h"
#include "../../include/cuzfp_hip.h"

namespace cuZFP {
namespace {

// pointers.cuh:12-22 (is_gpu_ptr): device or managed memory is used in place.
bool is_device_ptr(const void* p) {
  if (!p) return false;
  hipPointerAttribute_t a;
  const hipError_t e = hipPointerGetAttributes(&a, p);
  (void)hipGetLastError();  // host pointers report an error: clear it
  if (e != hipSuccess) return false;
  return a.type == hipMemoryTypeDevice || a.type == hipMemoryTypeManaged;
}

thread_local int t_last_status = CUZFP_SUCCESS;

void report(const char* what, int rc) {
  t_last_status = rc;
  std::fprintf(stderr, "cuZFP: %s failed: %s", what, cuzfp_hip_status_string(rc));
  if (rc == CUZFP_ERROR_HIP)
    std::fprintf(stderr, " (%s)", hipGetErrorString((hipError_t)cuzfp_hip_last_hip_error()));
  std::fprintf(stderr, "\n");
}

// Element span [lo, hi] touched by a (possibly strided) field, relative to data.
void field_span(const zfp_field* f, long long* lo, long long* hi) {
  const uint d = zfp_field_dimensionality(f);
  const long long nx = f->nx, ny = d > 1 ? f->ny : 1, nz = d > 2 ? f->nz : 1;
  const long long sx = f->sx ? f->sx : 1, sy = f->sy ? f->sy : nx, sz = f->sz ? f->sz : nx * ny;
  *lo = 0;
  *hi = 0;
  const long long ext[3][2] = {{sx, nx}, {sy, ny}, {sz, nz}};
  for (int i = 0; i < 3; i++) {
    const long long v = ext[i][0] * (ext[i][1] - 1);
    if (v < 0) *lo += v; else *hi += v;
  }
}

bool contiguous(const zfp_field* f) {
  const uint d = zfp_field_dimensionality(f);
  const long long nx = f->nx, ny = d > 1 ? f->ny : 1;
  return (!f->sx || f->sx == 1) && (!f->sy || f->sy == nx) && (!f->sz || f->sz == nx * ny);
}

struct DeviceField {
  void* base = nullptr;   // device allocation (null if used in place)
  void* data = nullptr;   // device pointer to element 0
  void* host = nullptr;   // host span start (for copy-back)
  size_t bytes = 0;
  ~DeviceField() { if (base) (void)hipFree(base); }
};

// setup_device_field (cuZFP.cu:124-155), generalised to strided spans.
int stage_field(zfp_field* f, bool upload, DeviceField* df) {
  if (is_device_ptr(f->data)) {
    df->data = f->data;
    return CUZFP_SUCCESS;
  }
  const size_t es = zfp_type_size(f->type);
  long long lo, hi;
  field_span(f, &lo, &hi);
  df->bytes = (size_t)(hi - lo + 1) * es;
  if (hipMalloc(&df->base, df->bytes) != hipSuccess) return CUZFP_ERROR_HIP;
  df->host = (char*)f->data + lo * (long long)es;
  df->data = (char*)df->base - lo * (long long)es;
  if (upload && hipMemcpy(df->base, df->host, df->bytes, hipMemcpyHostToDevice) != hipSuccess)
    return CUZFP_ERROR_HIP;
  return CUZFP_SUCCESS;
}

}  // namespace

size_t compress(zfp_stream* stream, zfp_field* field) {
  t_last_status = CUZFP_SUCCESS;
  if (!stream || !field || !stream->stream || !field->data) {
    report("compress", CUZFP_ERROR_INVALID_ARGUMENT);
    return 0;
  }
  const int type = (int)field->type;
  const uint nx = field->nx, ny = field->ny, nz = field->nz;
  const size_t need = cuzfp_hip_stream_bytes(type, nx, ny, nz, stream->maxbits);
  if (!need) {
    report("compress", CUZFP_ERROR_INVALID_ARGUMENT);
    return 0;
  }
  const bool dev_stream = is_device_ptr(stream->stream);
  const bool dev_field = is_device_ptr(field->data);
  int rc;
  size_t bytes = 0;
  if (!dev_stream && !dev_field && contiguous(field)) {
    rc = cuzfp_hip_compress_host(field->data, type, nx, ny, nz, stream->maxbits, stream->stream,
                                 need, &bytes, CUZFP_HOST_STREAMS);
    if (rc) report("compress", rc);
    return rc ? 0 : bytes;
  }
  DeviceField df;
  rc = stage_field(field, true, &df);
  uint64_t* d_stream = (uint64_t*)stream->stream;
  void* tmp = nullptr;
  if (!rc && !dev_stream) {
    if (hipMalloc(&tmp, need) != hipSuccess) rc = CUZFP_ERROR_HIP;
    d_stream = (uint64_t*)tmp;
  }
  if (!rc)
    rc = cuzfp_hip_encode(df.data, type, nx, ny, nz, field->sx, field->sy, field->sz,
                          stream->maxbits, d_stream, need, &bytes, 0);
  if (!rc && hipDeviceSynchronize() != hipSuccess) rc = CUZFP_ERROR_HIP;
  if (!rc && !dev_stream &&
      hipMemcpy(stream->stream, d_stream, bytes, hipMemcpyDeviceToHost) != hipSuccess)
    rc = CUZFP_ERROR_HIP;
  if (tmp) (void)hipFree(tmp);
  if (rc) {
    report("compress", rc);
    return 0;
  }
  return bytes;
}

void decompress(zfp_stream* stream, zfp_field* field) {
  t_last_status = CUZFP_SUCCESS;
  if (!stream || !field || !stream->stream || !field->data) {
    report("decompress", CUZFP_ERROR_INVALID_ARGUMENT);
    return;
  }
  const int type = (int)field->type;
  const uint nx = field->nx, ny = field->ny, nz = field->nz;
  const size_t need = cuzfp_hip_stream_bytes(type, nx, ny, nz, stream->maxbits);
  if (!need) {
    report("decompress", CUZFP_ERROR_INVALID_ARGUMENT);
    return;
  }
  const bool dev_stream = is_device_ptr(stream->stream);
  const bool dev_field = is_device_ptr(field->data);
  int rc;
  if (!dev_stream && !dev_field && contiguous(field)) {
    rc = cuzfp_hip_decompress_host(stream->stream, need, type, nx, ny, nz, stream->maxbits,
                                   field->data, CUZFP_HOST_STREAMS);
    if (rc) report("decompress", rc);
    return;
  }
  DeviceField df;
  // a strided host output must keep the elements between its rows: upload it
  rc = stage_field(field, !contiguous(field), &df);
  const uint64_t* d_stream = (const uint64_t*)stream->stream;
  void* tmp = nullptr;
  if (!rc && !dev_stream) {
    if (hipMalloc(&tmp, need) != hipSuccess ||
        hipMemcpy(tmp, stream->stream, need, hipMemcpyHostToDevice) != hipSuccess)
      rc = CUZFP_ERROR_HIP;
    d_stream = (const uint64_t*)tmp;
  }
  if (!rc)
    rc = cuzfp_hip_decode(d_stream, need, type, nx, ny, nz, field->sx, field->sy, field->sz,
                          stream->maxbits, df.data, 0);
  if (!rc && hipDeviceSynchronize() != hipSuccess) rc = CUZFP_ERROR_HIP;
  if (!rc && df.base && hipMemcpy(df.host, df.base, df.bytes, hipMemcpyDeviceToHost) != hipSuccess)
    rc = CUZFP_ERROR_HIP;
  if (tmp) (void)hipFree(tmp);
  if (rc) report("decompress", rc);
}

}  // namespace cuZFP

// extension: the status of this thread's last compress / decompress call
extern "C" int cuZFP_last_status(void) { return cuZFP::t_last_status; }
