// cuzfp_amd/cli/data_gen.cpp -- synthetic input arrays for the CLI fuzz harness.
//
// Same options and fields as the reference generator (src/utils/data_gen.cpp:9-232):
//   data_gen -o <file|-> [-t i32|i64|f32|f64 (default f64)] -1 nx | -2 nx ny | -3 nx ny nz
// 1D: a[x] = 10 sin(x * 3.14/180) (data_gen.cpp:29-39); 2D/3D: the "braid" field of
// sines and cosines over a[z][y][x] (data_gen.cpp:41-80), cast to the scalar type.
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

namespace {

[[noreturn]] void usage() {
  std::fprintf(stderr,
      "Usage: data_gen <options>\n"
      "Output:\n"
      "  -o <path> : binary output file (\"-\" for stdout)\n"
      "Array type and dimensions:\n"
      "  -t <i32|i64|f32|f64> : integer or floating scalar type (default = f64)\n"
      "  -1 <nx> : dimensions for 1D array a[nx]\n"
      "  -2 <nx> <ny> : dimensions for 2D array a[ny][nx]\n"
      "  -3 <nx> <ny> <nz> : dimensions for 3D array a[nz][ny][nx]\n");
  std::exit(EXIT_FAILURE);
}

double sine_1d(size_t x) { return std::sin((double)x * (3.14 / 180.)) * 10.0; }

double braid(unsigned x, unsigned y, unsigned z, unsigned nx, unsigned ny, unsigned nz) {
  const double dx = 4.0 * 3.14 / (double)(nx - 1), dy = 2.0 * 3.14 / (double)(ny - 1);
  const double dz = 3.0 * 3.14 / (double)(nz - 1);
  const double cx = x * dx + 2.0 * 3.14, cy = y * dy - 3.14;
  double v = std::sin(cx) + std::sin(cy);
  v += 2.0 * std::cos(std::sqrt(cx * cx / 2.0 + cy * cy) / .75);
  v += 4.0 * std::cos(cx * cy / 4.0);
  if (z > 1) {
    const double cz = z * dz - 1.5 * 3.14;
    v += std::sin(cz) + 1.5 * std::cos(std::sqrt(cx * cx + cy * cy + cz * cz) / 0.75);
  }
  return v;
}

template <typename T>
std::vector<unsigned char> generate(unsigned dims, unsigned nx, unsigned ny, unsigned nz) {
  const size_t n = (size_t)nx * ny * nz;
  std::vector<unsigned char> out(n * sizeof(T));
  T* a = (T*)out.data();
  if (dims == 1) {
    for (size_t x = 0; x < n; x++) a[x] = static_cast<T>(sine_1d(x));
  } else {
    size_t i = 0;
    for (unsigned z = 0; z < nz; z++)
      for (unsigned y = 0; y < ny; y++)
        for (unsigned x = 0; x < nx; x++) a[i++] = static_cast<T>(braid(x, y, z, nx, ny, nz));
  }
  return out;
}

}  // namespace

int main(int argc, char** argv) {
  unsigned dims = 0, nx = 0, ny = 1, nz = 1;
  const char* outpath = nullptr;
  const char* type = "f64";
  auto uarg = [&](int& i, unsigned& v) {
    if (++i == argc || std::sscanf(argv[i], "%u", &v) != 1) usage();
  };
  for (int i = 1; i < argc; i++) {
    if (argv[i][0] != '-' || !argv[i][1] || argv[i][2]) usage();
    switch (argv[i][1]) {
      case '1': uarg(i, nx); ny = nz = 1; dims = 1; break;
      case '2': uarg(i, nx); uarg(i, ny); nz = 1; dims = 2; break;
      case '3': uarg(i, nx); uarg(i, ny); uarg(i, nz); dims = 3; break;
      case 'o': if (++i == argc) usage(); outpath = argv[i]; break;
      case 't':
        if (++i == argc) usage();
        type = argv[i];
        if (std::strcmp(type, "i32") && std::strcmp(type, "i64") && std::strcmp(type, "f32") &&
            std::strcmp(type, "f64"))
          usage();
        break;
      default: usage();
    }
  }
  if (!dims || !outpath) usage();
  std::vector<unsigned char> data;
  if (!std::strcmp(type, "i32")) data = generate<int32_t>(dims, nx, ny, nz);
  else if (!std::strcmp(type, "i64")) data = generate<int64_t>(dims, nx, ny, nz);
  else if (!std::strcmp(type, "f32")) data = generate<float>(dims, nx, ny, nz);
  else data = generate<double>(dims, nx, ny, nz);
  FILE* f = !std::strcmp(outpath, "-") ? stdout : std::fopen(outpath, "wb");
  if (!f) {
    std::fprintf(stderr, "cannot create output file\n");
    return EXIT_FAILURE;
  }
  if (std::fwrite(data.data(), 1, data.size(), f) != data.size()) {
    std::fprintf(stderr, "cannot write output file\n");
    return EXIT_FAILURE;
  }
  if (f != stdout) std::fclose(f);
  return EXIT_SUCCESS;
}
