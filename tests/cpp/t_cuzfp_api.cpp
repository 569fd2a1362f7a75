// tests/cpp/t_cuzfp_api.cpp -- the reference's gtest programs, against the drop-in.
//
// Each TEST below restates one test of mclarsen/cuZFP src/tests/ through the
// unchanged C++ surface (include/cuZFP.h + zfp_structs.h, `using namespace
// cuZFP` as the reference tests do), linked against libcuZFP.so:
//   sanity_check_{1,2,3}  t_sanity_check_{1,2,3}.cpp  ramp f[i] = i at rate 8
//   encode_decode_{1,2,3} t_encode_decode_{1,2,3}.cpp sine / radial / 1/r fields
//   device_stream / host_stream  t_cuda_mem.cu        stream in device / host memory
// plus: device-resident field, strided field, and agreement of every staging
// path (host/host, host/device, device/device) byte for byte.  The reference's
// encode_decode tests only print errors; here the errors are asserted against
// the rate-8 bounds CPU zfp achieves on the same fields, and each stream is
// written to argv[1]/<name>.bin for tests/test_cpp_api.py to compare with the
// CPU oracle bit for bit (with its input <name>.in and output <name>.out).
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <functional>
#include <string>
#include <vector>

#include <cuZFP.h>

using namespace cuZFP;

static int g_failures = 0;
static std::string g_outdir = ".";
#define CHECK(c)                                                                  \
  do {                                                                            \
    if (!(c)) {                                                                   \
      std::printf("  FAILED %s:%d: %s\n", __FILE__, __LINE__, #c);                \
      g_failures++;                                                               \
      return;                                                                     \
    }                                                                             \
  } while (0)

static void save(const std::string& name, const void* p, size_t n) {
  FILE* f = std::fopen((g_outdir + "/" + name).c_str(), "wb");
  if (f) {
    std::fwrite(p, 1, n, f);
    std::fclose(f);
  }
}

template <typename T>
static std::vector<unsigned char> roundtrip(std::vector<T>& in, std::vector<T>& out, int nx, int ny,
                                            int nz, double rate, const char* name = nullptr) {
  zfp_stream zfp;
  const zfp_type type = get_zfp_type<T>();
  const uint dims = nz ? 3 : ny ? 2 : 1;
  zfp_field* field = dims == 3 ? zfp_field_3d(in.data(), type, nx, ny, nz)
                   : dims == 2 ? zfp_field_2d(in.data(), type, nx, ny)
                               : zfp_field_1d(in.data(), type, nx);
  stream_set_rate(&zfp, rate, type, dims);
  const size_t cap = zfp_stream_maximum_size(&zfp, field);
  std::vector<unsigned char> buffer(cap);
  zfp.stream = (Word*)buffer.data();
  const size_t bytes = compress(&zfp, field);
  zfp_field* out_field = dims == 3 ? zfp_field_3d(out.data(), type, nx, ny, nz)
                       : dims == 2 ? zfp_field_2d(out.data(), type, nx, ny)
                                   : zfp_field_1d(out.data(), type, nx);
  decompress(&zfp, out_field);
  zfp_field_free(out_field);
  zfp_field_free(field);
  buffer.resize(bytes);
  if (name) {  // input, stream and output for the oracle comparison
    save(std::string(name) + ".in", in.data(), in.size() * sizeof(T));
    save(std::string(name) + ".bin", buffer.data(), buffer.size());
    save(std::string(name) + ".out", out.data(), out.size() * sizeof(T));
  }
  return buffer;
}

// t_sanity_check_1.cpp: 1D ramp of 128 values at rate 8
static void sanity_check_1() {
  std::vector<float> a(128), b(128);
  for (int i = 0; i < 128; i++) a[i] = (float)i;
  auto s = roundtrip(a, b, 128, 0, 0, 8, "sanity_1");
  CHECK(s.size() == 128);
  for (int i = 0; i < 128; i++) CHECK(i == static_cast<int>(b[i]));
}

// t_sanity_check_2.cpp: 4 x 4 ramp (the reference's 2D launcher divides the
// grid by 128 twice, encode2.cuh:489-491, and encodes nothing here)
static void sanity_check_2() {
  std::vector<float> a(16), b(16);
  for (int i = 0; i < 16; i++) a[i] = (float)i;
  auto s = roundtrip(a, b, 4, 4, 0, 8, "sanity_2");
  CHECK(s.size() == 16);
  for (int i = 0; i < 16; i++) CHECK(i == static_cast<int>(b[i]));
}

// t_sanity_check_3.cpp: 16 x 8 x 4 ramp
static void sanity_check_3() {
  const int n = 16 * 8 * 4;
  std::vector<float> a(n), b(n);
  for (int i = 0; i < n; i++) a[i] = (float)i;
  auto s = roundtrip(a, b, 16, 8, 4, 8, "sanity_3");
  CHECK(s.size() == (size_t)(n / 64) * 64);
  for (int i = 0; i < n; i++) CHECK(i == static_cast<int>(b[i]));
}

template <typename T>
static double mean_abs_err(const std::vector<T>& a, const std::vector<T>& b) {
  double e = 0;
  for (size_t i = 0; i < a.size(); i++) e += std::fabs((double)a[i] - (double)b[i]);
  return e / (double)a.size();
}

// t_encode_decode_1.cpp: 10 sin(x deg), 256 values, rate 8
static void encode_decode_1() {
  const int nx = 256;
  std::vector<float> a(nx), b(nx);
  for (int x = 0; x < nx; x++) a[x] = (float)(std::sin(double(x) * (3.14 / 180.)) * 10.);
  auto s = roundtrip(a, b, nx, 0, 0, 8, "encode_decode_1");
  const double e = mean_abs_err(a, b);
  std::printf("  encode_decode_1 mean abs err %.3e\n", e);
  CHECK(e < 5e-2);  // CPU zfp: 1.7e-2
}

// t_encode_decode_2.cpp: sqrt(x^2 + y^2) on 4096 x 1024, rate 8
static void encode_decode_2() {
  const int nx = 4096, ny = 1024;
  std::vector<float> a((size_t)nx * ny), b((size_t)nx * ny);
  for (int y = 0; y < ny; y++)
    for (int x = 0; x < nx; x++) a[(size_t)y * nx + x] = (float)std::sqrt(double(x) * x + double(y) * y);
  auto s = roundtrip(a, b, nx, ny, 0, 8, "encode_decode_2");
  const double e = mean_abs_err(a, b);
  std::printf("  encode_decode_2 mean abs err %.3e\n", e);
  CHECK(e < 1e-4);  // CPU zfp: 7.3e-6
}

// t_encode_decode_3.cpp: 1/r on 256^3 (1 at the origin), rate 8
template <typename T>
static void encode_decode_3_t(const char* name, double bound) {
  const int n = 256;
  std::vector<T> a((size_t)n * n * n), b(a.size());
  for (int z = 0; z < n; z++)
    for (int y = 0; y < n; y++)
      for (int x = 0; x < n; x++) {
        T v = static_cast<T>(std::sqrt(double(z * z) + double(x * x) + double(y * y)));
        a[((size_t)z * n + y) * n + x] = v != 0 ? (T)(1. / v) : (T)1;
      }
  auto s = roundtrip(a, b, n, n, n, 8, name);
  const double e = mean_abs_err(a, b);
  std::printf("  %s mean abs err %.3e\n", name, e);
  CHECK(e < bound);
}
static void encode_decode_3() { encode_decode_3_t<float>("encode_decode_3", 1e-6); }
static void encode_decode_3_f64() { encode_decode_3_t<double>("encode_decode_3_f64", 1e-6); }

// t_cuda_mem.cu: the stream buffer lives in device memory (hipMalloc)
static void device_stream() {
  const int x = 16, y = 8, z = 4, n = x * y * z;
  std::vector<float> a(n), b(n);
  for (int i = 0; i < n; i++) a[i] = (float)i;
  zfp_stream zfp;
  zfp_field* field = zfp_field_3d(a.data(), zfp_type_float, x, y, z);
  stream_set_rate(&zfp, 8, field->type, 3);
  const size_t cap = zfp_stream_maximum_size(&zfp, field);
  Word* d_stream = nullptr;
  CHECK(hipMalloc(&d_stream, cap) == hipSuccess);
  zfp.stream = d_stream;
  const size_t bytes = compress(&zfp, field);
  zfp_field* out = zfp_field_3d(b.data(), zfp_type_float, x, y, z);
  decompress(&zfp, out);
  std::vector<unsigned char> host(bytes);
  CHECK(hipMemcpy(host.data(), d_stream, bytes, hipMemcpyDeviceToHost) == hipSuccess);
  save("device_stream.bin", host.data(), host.size());
  zfp_field_free(out);
  zfp_field_free(field);
  (void)hipFree(d_stream);
  CHECK(bytes == 512);
  for (int i = 0; i < n; i++) CHECK(i == static_cast<int>(b[i]));
}

// t_cuda_mem.cu t_host_mem_check
static void host_stream() {
  const int n = 16 * 8 * 4;
  std::vector<float> a(n), b(n);
  for (int i = 0; i < n; i++) a[i] = (float)i;
  auto s = roundtrip(a, b, 16, 8, 4, 8);
  for (int i = 0; i < n; i++) CHECK(i == static_cast<int>(b[i]));
}

// device-resident field and stream: no staging at all; same bytes as host path
static void device_field() {
  const int nx = 40, ny = 24, nz = 12, n = nx * ny * nz;
  std::vector<float> a(n), b(n);
  for (int i = 0; i < n; i++) a[i] = std::sin(0.01f * i) * 3.0f;
  auto ref = roundtrip(a, b, nx, ny, nz, 8);
  float *d_in = nullptr, *d_out = nullptr;
  Word* d_stream = nullptr;
  CHECK(hipMalloc(&d_in, n * 4) == hipSuccess);
  CHECK(hipMalloc(&d_out, n * 4) == hipSuccess);
  CHECK(hipMemcpy(d_in, a.data(), n * 4, hipMemcpyHostToDevice) == hipSuccess);
  zfp_stream zfp;
  zfp_field* field = zfp_field_3d(d_in, zfp_type_float, nx, ny, nz);
  stream_set_rate(&zfp, 8, zfp_type_float, 3);
  const size_t cap = zfp_stream_maximum_size(&zfp, field);
  CHECK(hipMalloc(&d_stream, cap) == hipSuccess);
  zfp.stream = d_stream;
  const size_t bytes = compress(&zfp, field);
  CHECK(bytes == ref.size());
  std::vector<unsigned char> got(bytes);
  CHECK(hipMemcpy(got.data(), d_stream, bytes, hipMemcpyDeviceToHost) == hipSuccess);
  CHECK(std::memcmp(got.data(), ref.data(), bytes) == 0);
  zfp_field* out = zfp_field_3d(d_out, zfp_type_float, nx, ny, nz);
  decompress(&zfp, out);
  std::vector<float> c(n);
  CHECK(hipMemcpy(c.data(), d_out, n * 4, hipMemcpyDeviceToHost) == hipSuccess);
  CHECK(std::memcmp(c.data(), b.data(), n * 4) == 0);
  zfp_field_free(out);
  zfp_field_free(field);
  (void)hipFree(d_in);
  (void)hipFree(d_out);
  (void)hipFree(d_stream);
}

// strided host field (every other z-plane of a bigger array): zfp honours
// sx/sy/sz (template/compress.c:246-291); cuZFP ignored them
static void strided_field() {
  const int nx = 20, ny = 12, nz = 8, NZ = 2 * nz;
  std::vector<double> big((size_t)nx * ny * NZ), out(big.size(), -1.0);
  for (size_t i = 0; i < big.size(); i++) big[i] = std::cos(0.003 * (double)i);
  std::vector<double> packed((size_t)nx * ny * nz), packed_out(packed.size());
  for (int z = 0; z < nz; z++)
    std::memcpy(&packed[(size_t)z * nx * ny], &big[(size_t)2 * z * nx * ny], sizeof(double) * nx * ny);
  auto ref = roundtrip(packed, packed_out, nx, ny, nz, 16);
  zfp_stream zfp;
  zfp_field* field = zfp_field_3d(big.data(), zfp_type_double, nx, ny, nz);
  field->sx = 1;
  field->sy = nx;
  field->sz = 2 * nx * ny;
  stream_set_rate(&zfp, 16, zfp_type_double, 3);
  std::vector<unsigned char> buf(zfp_stream_maximum_size(&zfp, field));
  zfp.stream = (Word*)buf.data();
  const size_t bytes = compress(&zfp, field);
  CHECK(bytes == ref.size());
  CHECK(std::memcmp(buf.data(), ref.data(), bytes) == 0);
  zfp_field* of = zfp_field_3d(out.data(), zfp_type_double, nx, ny, nz);
  of->sx = 1;
  of->sy = nx;
  of->sz = 2 * nx * ny;
  decompress(&zfp, of);
  for (int z = 0; z < nz; z++) {
    CHECK(std::memcmp(&out[(size_t)2 * z * nx * ny], &packed_out[(size_t)z * nx * ny],
                      sizeof(double) * nx * ny) == 0);
    if (z + 1 < nz) CHECK(out[(size_t)(2 * z + 1) * nx * ny] == -1.0);  // gaps untouched
  }
  zfp_field_free(of);
  zfp_field_free(field);
}

int main(int argc, char** argv) {
  if (argc > 1) g_outdir = argv[1];
  const std::vector<std::pair<const char*, std::function<void()>>> tests = {
      {"sanity_check_1", sanity_check_1}, {"sanity_check_2", sanity_check_2},
      {"sanity_check_3", sanity_check_3}, {"encode_decode_1", encode_decode_1},
      {"encode_decode_2", encode_decode_2}, {"encode_decode_3", encode_decode_3},
      {"encode_decode_3_f64", encode_decode_3_f64}, {"device_stream", device_stream},
      {"host_stream", host_stream}, {"device_field", device_field},
      {"strided_field", strided_field}};
  for (auto& t : tests) {
    const int before = g_failures;
    std::printf("[ RUN  ] %s\n", t.first);
    t.second();
    std::printf("[ %s ] %s\n", g_failures == before ? " OK " : "FAIL", t.first);
  }
  std::printf("%d failure(s)\n", g_failures);
  return g_failures ? 1 : 0;
}
