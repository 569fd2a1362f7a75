// cuzfp_amd/cli/cuda_zfp.cpp -- the `cuda_zfp` command-line codec on the MI355X library.
//
// Same options and file semantics as the reference CLI (src/utils/cuda_zfp.cpp:35-423),
// itself modelled on CPU zfp 0.5.0's `zfp` tool (zfp-0.5.0/utils/zfp.c):
//
//   -i <file>   raw input array          -z <file>   compressed output (with -i) or input
//   -o <file>   decompressed output      -s          error statistics    -q  quiet
//   -f | -d | -t <i32|i64|f32|f64>       -1 nx | -2 nx ny | -3 nx ny nz
//   -r <rate>   fixed rate (bits/value)  -c minbits maxbits maxprec minexp (fixed-rate form only)
//   -h          write / read zfp's 96- or 148-bit header (zfp.c:661-719)
//
// Compression and decompression run through cuZFP::compress / decompress (libcuZFP.so,
// host buffers staged through the GPU).  Streams are those of CPU zfp 0.5.0 for the
// same field and maxbits, byte for byte (tests/fuzz_cli.py diffs them against the
// reference's `zfp` tool, as src/utils/test.py:68-93 does).
//
// Differences from the reference CLI, all toward CPU zfp's tool: -h is honoured (the
// reference parses and ignores it); -s and the summary line are printed (a TODO in the
// reference, :417); -p/-a fail with a message, as the reference does (:342-346); a
// failed call exits non-zero instead of continuing.
#include <cuZFP.h>

#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

namespace {

using cuZFP::zfp_type;

[[noreturn]] void usage() {
  std::fprintf(stderr,
      "Usage: cuda_zfp <options>\n"
      "General options:\n"
      "  -h : read/write array and compression parameters from/to compressed header\n"
      "  -q : quiet mode; suppress output\n"
      "  -s : print error statistics\n"
      "Input and output:\n"
      "  -i <path> : uncompressed binary input file (\"-\" for stdin)\n"
      "  -o <path> : decompressed binary output file (\"-\" for stdout)\n"
      "  -z <path> : compressed input (w/o -i) or output file (\"-\" for stdin/stdout)\n"
      "Array type and dimensions (needed with -i):\n"
      "  -f : single precision (float type)\n"
      "  -d : double precision (double type)\n"
      "  -t <i32|i64|f32|f64> : integer or floating scalar type\n"
      "  -1 <nx> : dimensions for 1D array a[nx]\n"
      "  -2 <nx> <ny> : dimensions for 2D array a[ny][nx]\n"
      "  -3 <nx> <ny> <nz> : dimensions for 3D array a[nz][ny][nx]\n"
      "Compression parameters (needed with -i):\n"
      "  -r <rate> : fixed rate (# compressed bits per value)\n"
      "  -c <minbits> <maxbits> <maxprec> <minexp> : fixed rate given as minbits = maxbits\n"
      "Examples:\n"
      "  -i ifile -z zfile -t f32 -3 64 64 64 -r 8 : compress to zfile\n"
      "  -z zfile -o ofile -t f32 -3 64 64 64 -r 8 : decompress zfile\n"
      "  -i ifile -s -d -1 1000000 -r 16 : round trip in memory, print error statistics\n");
  std::exit(EXIT_FAILURE);
}

int fail(const char* msg) {
  std::fprintf(stderr, "%s\n", msg);
  return EXIT_FAILURE;
}

// ---- zfp 0.5.0 header (zfp.c:661-687): 32-bit magic, 52-bit field metadata,
// 12-bit (maxbits <= 2048) or 64-bit mode, bits LSB first in 64-bit words.
constexpr unsigned kMagicBits = 32, kMetaBits = 52, kShortModeBits = 12, kLongModeBits = 64;
constexpr uint64_t kShortModeMax = (1u << kShortModeBits) - 2;

struct BitOut {  // little-endian bit appender (the layout of bitstream.c:66-87)
  std::vector<uint64_t> w;
  size_t pos = 0;
  void put(uint64_t v, unsigned n) {
    if (n < 64) v &= (1ull << n) - 1;
    while (w.size() * 64 < pos + n) w.push_back(0);
    const unsigned sh = pos & 63;
    w[pos >> 6] |= v << sh;
    if (sh + n > 64) w[(pos >> 6) + 1] |= v >> (64 - sh);
    pos += n;
  }
};

uint64_t bits_at(const uint64_t* w, size_t nwords, size_t pos, unsigned n) {
  auto word = [&](size_t i) { return i < nwords ? w[i] : 0ull; };
  const unsigned sh = pos & 63;
  uint64_t v = word(pos >> 6) >> sh;
  if (sh && sh + n > 64) v |= word((pos >> 6) + 1) << (64 - sh);
  return n < 64 ? v & ((1ull << n) - 1) : v;
}

// zfp.c:158-180
uint64_t field_metadata(zfp_type type, unsigned dims, unsigned nx, unsigned ny, unsigned nz) {
  uint64_t meta = 0;
  if (dims == 1) meta = nx - 1;
  if (dims == 2) meta = ((uint64_t)(ny - 1) << 24) + (nx - 1);
  if (dims == 3) meta = ((((uint64_t)(nz - 1) << 16) + (ny - 1)) << 16) + (nx - 1);
  meta = (meta << 2) + (dims - 1);
  return (meta << 2) + ((unsigned)type - 1);
}

// zfp.c:305-345 for fixed-rate parameters: the 12-bit form needs maxbits <= 2048 and
// maxprec >= 64, so float and int32 fields (maxprec 32, zfp.c:380-403) take the 64-bit form
uint64_t stream_mode(const cuZFP::zfp_stream& z) {
  if (z.minbits == z.maxbits && z.maxbits >= 1 && z.maxbits <= 2048 && z.maxprec >= ZFP_MAX_PREC &&
      z.minexp <= ZFP_MIN_EXP)
    return z.maxbits - 1;
  const uint64_t minbits = std::min(z.minbits, 0x8000u) - 1, maxbits = std::min(z.maxbits, 0x8000u) - 1;
  const uint64_t maxprec = std::min(z.maxprec, 0x80u) - 1;
  const uint64_t minexp = (uint64_t)std::max(0, std::min(z.minexp + 16495, 0x7fff));
  return ((((((minexp << 7) + maxprec) << 15) + maxbits) << 15) + minbits) << 12 | 0xfffu;
}

// zfp.c:689-719; only fixed-rate modes are accepted (the codec has no other)
bool read_header(const uint64_t* w, size_t nwords, zfp_type& type, unsigned& dims, unsigned& nx,
                 unsigned& ny, unsigned& nz, cuZFP::zfp_stream& z, unsigned& hbits) {
  size_t p = 0;
  const char magic[3] = {'z', 'f', 'p'};
  for (int i = 0; i < 3; i++, p += 8)
    if (bits_at(w, nwords, p, 8) != (uint64_t)(unsigned char)magic[i]) return false;
  if (bits_at(w, nwords, p, 8) != 0x05) return false;  // ZFP_VERSION >> 4 (zfp.h:71)
  p += 8;
  uint64_t meta = bits_at(w, nwords, p, kMetaBits);
  p += kMetaBits;
  type = (zfp_type)((meta & 3u) + 1);
  meta >>= 2;
  dims = (unsigned)(meta & 3u) + 1;
  meta >>= 2;
  nx = ny = nz = 1;
  if (dims == 1) nx = (unsigned)(meta & 0xffffffffffffull) + 1;
  if (dims == 2) { nx = (unsigned)(meta & 0xffffff) + 1; ny = (unsigned)((meta >> 24) & 0xffffff) + 1; }
  if (dims == 3) {
    nx = (unsigned)(meta & 0xffff) + 1;
    ny = (unsigned)((meta >> 16) & 0xffff) + 1;
    nz = (unsigned)((meta >> 32) & 0xffff) + 1;
  }
  if (dims > 3) return false;
  uint64_t mode = bits_at(w, nwords, p, kShortModeBits);
  p += kShortModeBits;
  if (mode > kShortModeMax) {
    mode += bits_at(w, nwords, p, kLongModeBits - kShortModeBits) << kShortModeBits;
    p += kLongModeBits - kShortModeBits;
    mode >>= 12;
    z.minbits = (unsigned)(mode & 0x7fff) + 1;
    z.maxbits = (unsigned)((mode >> 15) & 0x7fff) + 1;
    z.maxprec = (unsigned)((mode >> 30) & 0x7f) + 1;
    z.minexp = (int)((mode >> 37) & 0x7fff) - 16495;
    if (z.minbits != z.maxbits) return false;
  } else {
    if (mode >= 2048) return false;  // fixed precision / accuracy
    z.minbits = z.maxbits = (unsigned)mode + 1;
    z.maxprec = ZFP_MAX_PREC;
    z.minexp = ZFP_MIN_EXP;
  }
  hbits = (unsigned)p;
  return true;
}

FILE* open_file(const char* path, bool write) {
  if (!std::strcmp(path, "-")) return write ? stdout : stdin;
  return std::fopen(path, write ? "wb" : "rb");
}

bool read_all(const char* path, std::vector<unsigned char>& out) {
  FILE* f = open_file(path, false);
  if (!f) return false;
  unsigned char buf[1 << 16];
  size_t n;
  while ((n = std::fread(buf, 1, sizeof buf, f)) > 0) out.insert(out.end(), buf, buf + n);
  const bool ok = !std::ferror(f);
  if (f != stdin) std::fclose(f);
  return ok;
}

bool write_all(const char* path, const void* p, size_t n) {
  FILE* f = open_file(path, true);
  if (!f) return false;
  const bool ok = std::fwrite(p, 1, n, f) == n;
  if (f != stdout) std::fclose(f);
  return ok;
}

template <typename T>
void error_stats(const T* f, const T* g, size_t n) {  // zfp.c:28-57
  double fmin = (double)f[0], fmax = fmin, erms = 0, emax = 0;
  for (size_t i = 0; i < n; i++) {
    const double d = std::fabs((double)f[i] - (double)g[i]);
    emax = std::max(emax, d);
    erms += d * d;
    fmin = std::min(fmin, (double)f[i]);
    fmax = std::max(fmax, (double)f[i]);
  }
  erms = std::sqrt(erms / (double)n);
  const double nrmse = erms / (fmax - fmin), psnr = 20 * std::log10((fmax - fmin) / (2 * erms));
  std::fprintf(stderr, " rmse=%.4g nrmse=%.4g maxe=%.4g psnr=%.2f", erms, nrmse, emax, psnr);
}

const char* type_name(zfp_type t) {
  switch (t) {
    case cuZFP::zfp_type_int32: return "int32";
    case cuZFP::zfp_type_int64: return "int64";
    case cuZFP::zfp_type_float: return "float";
    default: return "double";
  }
}

}  // namespace

int main(int argc, char** argv) {
  zfp_type type = cuZFP::zfp_type_none;
  unsigned dims = 0, nx = 0, ny = 0, nz = 0;
  double rate = 0;
  unsigned minbits = 0, maxbits = 0, maxprec = 0;
  int minexp = ZFP_MIN_EXP;
  bool header = false, quiet = false, stats = false;
  const char *inpath = nullptr, *zfppath = nullptr, *outpath = nullptr;
  char mode = 0;

  if (argc == 1) usage();
  auto uarg = [&](int& i, unsigned& v) {
    if (++i == argc || std::sscanf(argv[i], "%u", &v) != 1) usage();
  };
  for (int i = 1; i < argc; i++) {
    if (argv[i][0] != '-' || !argv[i][1] || argv[i][2]) usage();
    switch (argv[i][1]) {
      case '1': uarg(i, nx); ny = nz = 1; dims = 1; break;
      case '2': uarg(i, nx); uarg(i, ny); nz = 1; dims = 2; break;
      case '3': uarg(i, nx); uarg(i, ny); uarg(i, nz); dims = 3; break;
      case 'a': case 'p':
        if (++i == argc) usage();
        mode = argv[i - 1][1];
        break;
      case 'c':
        uarg(i, minbits); uarg(i, maxbits); uarg(i, maxprec);
        if (++i == argc || std::sscanf(argv[i], "%d", &minexp) != 1) usage();
        mode = 'c';
        break;
      case 'd': type = cuZFP::zfp_type_double; break;
      case 'f': type = cuZFP::zfp_type_float; break;
      case 'h': header = true; break;
      case 'i': if (++i == argc) usage(); inpath = argv[i]; break;
      case 'o': if (++i == argc) usage(); outpath = argv[i]; break;
      case 'q': quiet = true; break;
      case 'r':
        if (++i == argc || std::sscanf(argv[i], "%lf", &rate) != 1) usage();
        mode = 'r';
        break;
      case 's': stats = true; break;
      case 't':
        if (++i == argc) usage();
        if (!std::strcmp(argv[i], "i32")) type = cuZFP::zfp_type_int32;
        else if (!std::strcmp(argv[i], "i64")) type = cuZFP::zfp_type_int64;
        else if (!std::strcmp(argv[i], "f32")) type = cuZFP::zfp_type_float;
        else if (!std::strcmp(argv[i], "f64")) type = cuZFP::zfp_type_double;
        else usage();
        break;
      case 'z': if (++i == argc) usage(); zfppath = argv[i]; break;
      default: usage();
    }
  }

  // the checks of cuda_zfp.cpp:230-268 / zfp.c:224-258
  if (!inpath && !zfppath) return fail("must specify uncompressed or compressed input file via -i or -z");
  if ((inpath || !header) && !cuZFP::zfp_type_size(type))
    return fail("must specify scalar type via -f, -d, or -t or header via -h");
  if ((inpath || !header) && !dims) return fail("must specify array dimensions via -1, -2, or -3 or header via -h");
  if ((inpath || !header) && !mode) return fail("must specify compression parameters via -a, -c, -p, or -r or header via -h");
  if (stats && !inpath) return fail("must specify input file via -i to compute stats");
  if (!inpath && zfppath && header && (cuZFP::zfp_type_size(type) || dims))
    return fail("cannot specify both field type/size and header");

  cuZFP::zfp_stream zfp{};
  if (inpath || !header) {
    if (mode == 'a' || mode == 'p') return fail("Currently, only the fixed rate '-r' mode is supported with CUDA");
    if (mode == 'r') {
      cuZFP::stream_set_rate(&zfp, rate, type, dims);
      zfp.maxprec = cuZFP::type_precision(type);  // as CPU zfp_stream_set_rate (zfp.c:380-403)
    } else {  // -c: the fixed-rate subset (zfp.c:336-345, zfp_stream_mode's first case)
      if (!maxbits) maxbits = ZFP_MAX_BITS;
      if (minbits != maxbits || (maxprec && maxprec < cuZFP::type_precision(type)) || minexp > ZFP_MIN_EXP)
        return fail("only fixed-rate parameters (minbits = maxbits, full precision) are supported");
      zfp.minbits = zfp.maxbits = maxbits;
      zfp.maxprec = maxprec ? maxprec : cuZFP::type_precision(type);
      zfp.minexp = ZFP_MIN_EXP;
    }
  }

  std::vector<unsigned char> raw_in;
  std::vector<unsigned char> packed;  // the file image of the compressed stream
  std::vector<Word> words;            // word-aligned stream handed to the codec
  size_t zfpsize = 0;

  auto fill_field = [&](cuZFP::zfp_field& f, void* data) {
    f.type = type;
    f.nx = nx;
    f.ny = dims >= 2 ? ny : 0;
    f.nz = dims >= 3 ? nz : 0;
    f.sx = f.sy = f.sz = 0;
    f.data = data;
  };
  const size_t count = (size_t)nx * (dims >= 2 ? ny : 1) * (dims >= 3 ? nz : 1);

  if (inpath) {
    if (!read_all(inpath, raw_in)) return fail("cannot open input file");
    if (raw_in.size() < count * cuZFP::zfp_type_size(type)) return fail("cannot read input file");
    cuZFP::zfp_field field;
    fill_field(field, raw_in.data());
    words.assign(cuZFP::zfp_stream_maximum_size(&zfp, &field) / 8 + 1, 0);
    zfp.stream = words.data();
    const size_t bytes = cuZFP::compress(&zfp, &field);
    if (!bytes) return fail("compression failed");
    if (header) {  // zfp_write_header + the stream after it, flushed to a word (zfp.c:661-687)
      BitOut out;
      out.put('z', 8); out.put('f', 8); out.put('p', 8); out.put(0x05, 8);
      out.put(field_metadata(type, dims, nx, ny, nz), kMetaBits);
      const uint64_t m = stream_mode(zfp);
      out.put(m, m > kShortModeMax ? kLongModeBits : kShortModeBits);
      // the payload is blocks x maxbits bits; the codec pads only its last word
      const size_t payload = (size_t)((nx + 3) / 4) * (dims >= 2 ? (ny + 3) / 4 : 1) *
                             (dims >= 3 ? (nz + 3) / 4 : 1) * (size_t)zfp.maxbits;
      for (size_t p = 0; p < payload; p += 64) {
        const unsigned n = (unsigned)std::min<size_t>(64, payload - p);
        out.put(bits_at((const uint64_t*)words.data(), words.size(), p, n), n);
      }
      zfpsize = ((out.pos + 63) / 64) * 8;
      out.w.resize(zfpsize / 8, 0);
      packed.assign((unsigned char*)out.w.data(), (unsigned char*)out.w.data() + zfpsize);
    } else {
      zfpsize = bytes;
      packed.assign((unsigned char*)words.data(), (unsigned char*)words.data() + zfpsize);
    }
    if (zfppath && !write_all(zfppath, packed.data(), zfpsize)) return fail("cannot write compressed file");
  } else {
    if (!read_all(zfppath, packed)) return fail("cannot open compressed file");
    zfpsize = packed.size();
  }

  std::vector<unsigned char> raw_out;
  if ((!inpath && zfppath) || outpath || stats) {
    const size_t nw = (packed.size() + 7) / 8;
    std::vector<uint64_t> file_words(nw + 1, 0);
    std::memcpy(file_words.data(), packed.data(), packed.size());
    unsigned hbits = 0;
    if (header) {
      if (!read_header(file_words.data(), nw, type, dims, nx, ny, nz, zfp, hbits))
        return fail("incorrect or missing header");
    }
    const size_t n = (size_t)nx * (dims >= 2 ? ny : 1) * (dims >= 3 ? nz : 1);
    const size_t blocks = (size_t)((nx + 3) / 4) * (dims >= 2 ? (ny + 3) / 4 : 1) * (dims >= 3 ? (nz + 3) / 4 : 1);
    const size_t payload = blocks * (size_t)zfp.maxbits;
    if ((size_t)hbits + payload > nw * 64) return fail("cannot read compressed file");
    words.assign((payload + 63) / 64 + 1, 0);
    for (size_t p = 0; p < payload; p += 64) {  // drop the header: blocks start at bit 0
      const unsigned k = (unsigned)std::min<size_t>(64, payload - p);
      words[p / 64] = bits_at(file_words.data(), nw, hbits + p, k);
    }
    raw_out.assign(n * cuZFP::zfp_type_size(type), 0);
    cuZFP::zfp_field field;
    fill_field(field, raw_out.data());
    zfp.stream = words.data();
    cuZFP::decompress(&zfp, &field);
    if (cuZFP_last_status()) return fail("decompression failed");
    if (outpath && !write_all(outpath, raw_out.data(), raw_out.size())) return fail("cannot write output file");
  }

  if (!quiet) {  // the summary line of zfp.c:463-469
    const size_t n = (size_t)nx * (dims >= 2 ? ny : 1) * (dims >= 3 ? nz : 1);
    const size_t rawsize = n * cuZFP::zfp_type_size(type);
    std::fprintf(stderr, "type=%s nx=%u ny=%u nz=%u", type_name(type), nx, dims >= 2 ? ny : 1, dims >= 3 ? nz : 1);
    std::fprintf(stderr, " raw=%lu zfp=%lu ratio=%.3g rate=%.4g", (unsigned long)rawsize, (unsigned long)zfpsize,
                 (double)rawsize / (double)zfpsize, 8.0 * (double)zfpsize / (double)n);
    if (stats) {
      switch (type) {
        case cuZFP::zfp_type_float: error_stats((const float*)raw_in.data(), (const float*)raw_out.data(), n); break;
        case cuZFP::zfp_type_double: error_stats((const double*)raw_in.data(), (const double*)raw_out.data(), n); break;
        case cuZFP::zfp_type_int32: error_stats((const int32_t*)raw_in.data(), (const int32_t*)raw_out.data(), n); break;
        default: error_stats((const int64_t*)raw_in.data(), (const int64_t*)raw_out.data(), n); break;
      }
    }
    std::fprintf(stderr, "\n");
  }
  return EXIT_SUCCESS;
}
