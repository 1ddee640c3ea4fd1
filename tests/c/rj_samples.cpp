/*
 * rj_samples.cpp -- this repository's restatement of the reference's three sample programs, so
 * that the reference's own CTest command lines (samples/CMakeLists.txt:25-179) run against the
 * drop-in library.  The reference samples themselves are not compiled here (DESIGN.md section 3
 * records why); this file follows their documented behaviour:
 *   - command line (samples/rocjpeg_samples_utils.h:89-179): -i <file|dir> -o <file|dir>
 *     -d <device> -be <backend> -fmt native|yuv_planar|y|rgb|rgb_planar -crop l,t,r,b
 *     -b <batch> -t <threads>;
 *   - destination sizing per output format and subsampling (rocjpeg_samples_utils.h:318-399),
 *     including its ROI rules;
 *   - the raw dump written by -o (rocjpeg_samples_utils.h:479-628): per channel, rows of the
 *     visible width read from the caller's pitch; for a directory input one file per image named
 *     <name>_<W>x<H>_<format>.<ext> (rocjpeg_samples_utils.h:420-470);
 *   - skip rules for a directory input (unparsable streams, < 64 px, 4:1:1 / unknown
 *     subsampling; jpegdecode.cpp:98-141), fatal for a single file.
 * Built three times (tests/c/Makefile) as jpegdecode_rj (one rocJpegDecode per image,
 * jpegdecode.cpp:72-163), jpegdecodebatched_rj (rocJpegDecodeBatched of -b images,
 * jpegdecodebatched.cpp:82-194) and jpegdecodeperf_rj (-t threads, each with its own handle,
 * batches of -b, jpegdecodeperf.cpp:75-158,228-271), linked with -lrocjpeg: the binaries carry
 * DT_NEEDED librocjpeg.so.0, as a binary built against rocJPEG does.  Exit code 0 = success.
 */
#include <hip/hip_runtime_api.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <dirent.h>
#include <string>
#include <sys/stat.h>
#include <thread>
#include <vector>

#include "rocjpeg.h"

#ifndef RJ_SAMPLE_MODE
#define RJ_SAMPLE_MODE 0  // 0 jpegdecode, 1 jpegdecodebatched, 2 jpegdecodeperf
#endif

namespace {

struct Args {
  std::string in, out;
  bool save = false;
  int device = 0, threads = 1, batch = 1;
  int passes = 1;  // jpegdecodeperf_rj only (not a reference option): timed passes over the thread's images
  RocJpegBackend backend = ROCJPEG_BACKEND_HARDWARE;
  RocJpegDecodeParams params{};
};

[[noreturn]] void Usage(const char *bad) {
  std::fprintf(stderr, "bad or incomplete option: %s\nusage: -i <file|dir> [-o out] [-d dev] [-be backend] "
                       "[-fmt native|yuv_planar|y|rgb|rgb_planar] [-crop l,t,r,b] [-b batch] [-t threads] [-n passes]\n",
               bad ? bad : "");
  std::exit(1);
}

Args Parse(int argc, char **argv) {
  Args a;
  a.params.output_format = ROCJPEG_OUTPUT_NATIVE;
  if (argc <= 1) Usage("");
  for (int i = 1; i < argc; i++) {
    const std::string o = argv[i];
    auto val = [&]() -> const char * {
      if (++i >= argc) Usage(o.c_str());
      return argv[i];
    };
    if (o == "-i") a.in = val();
    else if (o == "-o") { a.out = val(); a.save = true; }
    else if (o == "-d") a.device = std::atoi(val());
    else if (o == "-be") a.backend = RocJpegBackend(std::atoi(val()));
    else if (o == "-t") {
      a.threads = std::atoi(val());
      if (a.threads <= 0 || a.threads > 32) Usage(argv[i]);
    } else if (o == "-b") a.batch = std::max(1, std::atoi(val()));
    else if (o == "-n") a.passes = std::max(1, std::atoi(val()));
    else if (o == "-fmt") {
      const std::string f = val();
      if (f == "native") a.params.output_format = ROCJPEG_OUTPUT_NATIVE;
      else if (f == "yuv_planar") a.params.output_format = ROCJPEG_OUTPUT_YUV_PLANAR;
      else if (f == "y") a.params.output_format = ROCJPEG_OUTPUT_Y;
      else if (f == "rgb") a.params.output_format = ROCJPEG_OUTPUT_RGB;
      else if (f == "rgb_planar") a.params.output_format = ROCJPEG_OUTPUT_RGB_PLANAR;
      else Usage(f.c_str());
    } else if (o == "-crop") {
      RocJpegDecodeParams &p = a.params;
      if (std::sscanf(val(), "%hd,%hd,%hd,%hd", &p.crop_rectangle.left, &p.crop_rectangle.top, &p.crop_rectangle.right,
                      &p.crop_rectangle.bottom) != 4)
        Usage("-crop");
      if ((p.crop_rectangle.right - p.crop_rectangle.left) % 2 || (p.crop_rectangle.bottom - p.crop_rectangle.top) % 2) {
        std::printf("output crop rectangle must have width and height of even numbers\n");
        std::exit(1);
      }
    } else Usage(o.c_str());
  }
  if (a.in.empty()) Usage("-i");
  return a;
}

bool IsDir(const std::string &p) {
  struct stat st;
  return stat(p.c_str(), &st) == 0 && S_ISDIR(st.st_mode);
}

std::vector<std::string> Files(const std::string &in, bool &is_dir) {
  std::vector<std::string> f;
  is_dir = IsDir(in);
  if (!is_dir) {
    f.push_back(in);
    return f;
  }
  if (DIR *d = opendir(in.c_str())) {
    while (dirent *e = readdir(d)) {
      const std::string n = e->d_name;
      if (n == "." || n == "..") continue;
      const std::string p = in + "/" + n;
      if (!IsDir(p)) f.push_back(p);
    }
    closedir(d);
  }
  std::sort(f.begin(), f.end());  // the reference iterates in directory order; sorted here for a stable dump set
  return f;
}

bool ReadFile(const std::string &p, std::vector<unsigned char> &b) {
  FILE *fp = std::fopen(p.c_str(), "rb");
  if (!fp) return false;
  std::fseek(fp, 0, SEEK_END);
  const long n = std::ftell(fp);
  std::fseek(fp, 0, SEEK_SET);
  b.resize(size_t(n));
  const bool ok = std::fread(b.data(), 1, size_t(n), fp) == size_t(n);
  std::fclose(fp);
  return ok;
}

// One image's destination as the samples size it: visible size (the ROI when it is valid),
// per channel pitch, allocation bytes, and the rows x bytes the dump writes.
struct Dest {
  uint32_t n = 0, w = 0, h = 0;
  uint32_t pitch[4] = {}, alloc[4] = {}, dump_w[4] = {}, dump_h[4] = {};
};

constexpr uint32_t kRgbAlign = 4u << 20;  // the samples align RGB channel allocations to 4 MB
uint32_t AlignUp(uint32_t v, uint32_t a) { return (v + a - 1) / a * a; }

bool Size(const RocJpegDecodeParams &p, RocJpegChromaSubsampling css, const uint32_t *W, const uint32_t *H, Dest &d) {
  const int rw = p.crop_rectangle.right - p.crop_rectangle.left, rh = p.crop_rectangle.bottom - p.crop_rectangle.top;
  const bool roi = rw > 0 && rh > 0 && uint32_t(rw) <= W[0] && uint32_t(rh) <= H[0];
  const uint32_t w = roi ? uint32_t(rw) : W[0], h = roi ? uint32_t(rh) : H[0];
  d = Dest{};
  d.w = w;
  d.h = h;
  auto ch = [&](int c, uint32_t pitch, uint32_t rows_alloc, uint32_t dw, uint32_t dh) {
    d.pitch[c] = pitch;
    d.alloc[c] = pitch * rows_alloc;
    d.dump_w[c] = dw;
    d.dump_h[c] = dh;
  };
  switch (p.output_format) {
    case ROCJPEG_OUTPUT_NATIVE:
      switch (css) {
        case ROCJPEG_CSS_444: d.n = 3; for (int c = 0; c < 3; c++) ch(c, w, h, w, h); break;
        case ROCJPEG_CSS_440: d.n = 3; ch(0, w, h, w, h); ch(1, w, h >> 1, w, h >> 1); ch(2, w, h >> 1, w, h >> 1); break;
        case ROCJPEG_CSS_422: d.n = 1; ch(0, 2 * w, h, 2 * w, h); break;
        case ROCJPEG_CSS_420: d.n = 2; ch(0, w, h, w, h); ch(1, w, h >> 1, w, h >> 1); break;
        case ROCJPEG_CSS_400: d.n = 1; ch(0, w, h, w, h); break;
        default: return false;
      }
      break;
    case ROCJPEG_OUTPUT_YUV_PLANAR:
      if (css == ROCJPEG_CSS_400) {
        d.n = 1;
        ch(0, w, h, w, h);
      } else {
        // the samples' pitches: the ROI width for every plane, else the plane widths; rows: the
        // plane heights of GetImageInfo (rocjpeg_samples_utils.h:361-371)
        d.n = 3;
        const bool hs = css == ROCJPEG_CSS_422 || css == ROCJPEG_CSS_420, vs = css == ROCJPEG_CSS_440 || css == ROCJPEG_CSS_420;
        for (int c = 0; c < 3; c++) {
          const uint32_t pitch = roi ? w : W[c];
          const uint32_t dw = c == 0 ? w : (hs ? w >> 1 : w), dh = c == 0 ? h : (vs ? h >> 1 : h);
          ch(c, pitch, roi ? h : H[c], dw, dh);
        }
      }
      break;
    case ROCJPEG_OUTPUT_Y: d.n = 1; ch(0, w, h, w, h); break;
    case ROCJPEG_OUTPUT_RGB:
      d.n = 1;
      ch(0, 3 * w, h, 3 * w, h);
      d.alloc[0] = AlignUp(d.alloc[0], kRgbAlign);
      break;
    case ROCJPEG_OUTPUT_RGB_PLANAR:
      d.n = 3;
      for (int c = 0; c < 3; c++) {
        ch(c, w, h, w, h);
        d.alloc[c] = AlignUp(d.alloc[c], kRgbAlign);
      }
      break;
    default: return false;
  }
  return true;
}

std::string OutName(const std::string &dir, const std::string &file, RocJpegOutputFormat f, RocJpegChromaSubsampling css,
                    uint32_t w, uint32_t h) {
  std::string base = file.substr(file.find_last_of('/') + 1);
  base = base.substr(0, base.find_last_of('.'));
  std::string desc, ext = "yuv";
  switch (f) {
    case ROCJPEG_OUTPUT_NATIVE:
      desc = css == ROCJPEG_CSS_444 ? "444" : css == ROCJPEG_CSS_440 ? "440" : css == ROCJPEG_CSS_422 ? "422_yuyv"
           : css == ROCJPEG_CSS_420 ? "nv12" : "400";
      break;
    case ROCJPEG_OUTPUT_YUV_PLANAR: desc = "planar"; break;
    case ROCJPEG_OUTPUT_Y: desc = "400"; break;
    case ROCJPEG_OUTPUT_RGB: desc = "packed"; ext = "rgb"; break;
    case ROCJPEG_OUTPUT_RGB_PLANAR: desc = "planar"; ext = "rgb"; break;
    default: break;
  }
  return dir + "/" + base + "_" + std::to_string(w) + "x" + std::to_string(h) + "_" + desc + "." + ext;
}

bool Dump(const std::string &path, const Dest &d, const RocJpegImage &img) {
  FILE *fp = std::fopen(path.c_str(), "wb");
  if (!fp) return false;
  bool ok = true;
  std::vector<uint8_t> host;
  for (uint32_t c = 0; c < d.n && ok; c++) {
    if (img.channel[c] == nullptr || d.pitch[c] == 0) continue;
    const size_t bytes = size_t(d.pitch[c]) * d.dump_h[c];
    host.resize(bytes);
    ok = hipMemcpy(host.data(), img.channel[c], bytes, hipMemcpyDeviceToHost) == hipSuccess;
    for (uint32_t r = 0; ok && r < d.dump_h[c]; r++)
      ok = std::fwrite(host.data() + size_t(r) * d.pitch[c], 1, d.dump_w[c], fp) == d.dump_w[c];
  }
  std::fclose(fp);
  return ok;
}

#define CHECK_RJ(call)                                                                         \
  do {                                                                                         \
    const RocJpegStatus st_ = (call);                                                          \
    if (st_ != ROCJPEG_STATUS_SUCCESS) {                                                       \
      std::fprintf(stderr, "%s: %s (%d)\n", #call, rocJpegGetErrorName(st_), int(st_));        \
      return 1;                                                                                \
    }                                                                                          \
  } while (0)

// An image ready to decode: its bytes, parsed stream, destination.
struct Item {
  std::string path;
  std::vector<unsigned char> data;
  RocJpegStreamHandle s = nullptr;
  RocJpegChromaSubsampling css = ROCJPEG_CSS_UNKNOWN;
  Dest d;
  RocJpegImage img{};
};

void Free(Item &it) {
  for (int c = 0; c < 4; c++)
    if (it.img.channel[c]) (void)hipFree(it.img.channel[c]);
  it.img = RocJpegImage{};
  if (it.s) (void)rocJpegStreamDestroy(it.s);
  it.s = nullptr;
}

// Parse + info + destination of one file.  1: skipped (directory input), 0: ready, -1: fatal.
int Prepare(RocJpegHandle h, const Args &a, bool is_dir, Item &it) {
  if (!ReadFile(it.path, it.data)) {
    std::fprintf(stderr, "cannot read %s\n", it.path.c_str());
    return -1;
  }
  if (rocJpegStreamCreate(&it.s) != ROCJPEG_STATUS_SUCCESS) return -1;
  const RocJpegStatus ps = rocJpegStreamParse(it.data.data(), it.data.size(), it.s);
  if (ps != ROCJPEG_STATUS_SUCCESS) {
    std::fprintf(stderr, "%s: parse failed: %s\n", it.path.c_str(), rocJpegGetErrorName(ps));
    return is_dir ? 1 : -1;
  }
  uint8_t nc = 0;
  uint32_t W[4] = {}, H[4] = {};
  if (rocJpegGetImageInfo(h, it.s, &nc, &it.css, W, H) != ROCJPEG_STATUS_SUCCESS) return -1;
  if (W[0] < 64 || H[0] < 64 || it.css == ROCJPEG_CSS_411 || it.css == ROCJPEG_CSS_UNKNOWN) {
    std::fprintf(stderr, "%s: unsupported (%ux%u, css %d)\n", it.path.c_str(), W[0], H[0], int(it.css));
    return is_dir ? 1 : -1;
  }
  if (!Size(a.params, it.css, W, H, it.d)) return -1;
  for (uint32_t c = 0; c < it.d.n; c++) {
    if (hipMalloc(reinterpret_cast<void **>(&it.img.channel[c]), it.d.alloc[c]) != hipSuccess) return -1;
    it.img.pitch[c] = it.d.pitch[c];
  }
  return 0;
}

int Save(const Args &a, bool is_dir, const Item &it) {
  if (!a.save) return 0;
  const std::string p = is_dir ? OutName(a.out, it.path, a.params.output_format, it.css, it.d.w, it.d.h) : a.out;
  if (!Dump(p, it.d, it.img)) {
    std::fprintf(stderr, "cannot write %s\n", p.c_str());
    return 1;
  }
  return 0;
}

// jpegdecode / jpegdecodebatched: one handle, files in order, -b images per call (batched mode).
int RunSerial(const Args &a, bool batched) {
  bool is_dir = false;
  const std::vector<std::string> files = Files(a.in, is_dir);
  if (files.empty()) return 1;
  if (hipSetDevice(a.device) != hipSuccess) return 1;
  RocJpegHandle h = nullptr;
  CHECK_RJ(rocJpegCreate(a.backend, a.device, &h));
  const size_t per = batched ? size_t(a.batch) : 1u;
  size_t decoded = 0, skipped = 0;
  double ms = 0;
  for (size_t i = 0; i < files.size(); i += per) {
    std::vector<Item> items;
    for (size_t j = i; j < std::min(files.size(), i + per); j++) {
      Item it;
      it.path = files[j];
      const int r = Prepare(h, a, is_dir, it);
      if (r < 0) return 1;
      if (r > 0) {
        Free(it);
        skipped++;
        continue;
      }
      items.push_back(std::move(it));
    }
    if (items.empty()) continue;
    std::vector<RocJpegStreamHandle> hs;
    std::vector<RocJpegImage> imgs;
    for (auto &it : items) {
      hs.push_back(it.s);
      imgs.push_back(it.img);
    }
    const auto t0 = std::chrono::steady_clock::now();
    if (batched) CHECK_RJ(rocJpegDecodeBatched(h, hs.data(), int(hs.size()), &a.params, imgs.data()));
    else CHECK_RJ(rocJpegDecode(h, hs[0], &a.params, imgs.data()));
    ms += std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    for (auto &it : items) {
      if (Save(a, is_dir, it)) return 1;
      Free(it);
      decoded++;
    }
  }
  CHECK_RJ(rocJpegDestroy(h));
  std::printf("decoded %zu image(s), skipped %zu, %.3f ms per image\n", decoded, skipped, decoded ? ms / double(decoded) : 0.0);
  return decoded ? 0 : 1;
}

// jpegdecodeperf: -t threads, each with its own handle and its share of the files, batches of -b,
// images/s summed over the threads (jpegdecodeperf.cpp:268-271).
int RunPerf(const Args &a) {
  bool is_dir = false;
  const std::vector<std::string> files = Files(a.in, is_dir);
  if (files.empty()) return 1;
  if (hipSetDevice(a.device) != hipSuccess) return 1;
  std::vector<double> rate(size_t(a.threads), 0.0);
  std::atomic<int> fails{0};
  std::vector<std::thread> th;
  for (int t = 0; t < a.threads; t++)
    th.emplace_back([&, t]() {
      if (hipSetDevice(a.device) != hipSuccess) { fails++; return; }
      RocJpegHandle h = nullptr;
      if (rocJpegCreate(a.backend, a.device, &h) != ROCJPEG_STATUS_SUCCESS) { fails++; return; }
      std::vector<Item> items;
      for (size_t j = size_t(t); j < files.size(); j += size_t(a.threads)) {
        Item it;
        it.path = files[j];
        const int r = Prepare(h, a, is_dir, it);
        if (r < 0) { fails++; Free(it); break; }
        if (r > 0) { Free(it); continue; }
        items.push_back(std::move(it));
      }
      double ms = 0;
      size_t n = 0;
      for (int pass = 0; pass < a.passes; pass++)
      for (size_t i = 0; i < items.size(); i += size_t(a.batch)) {
        std::vector<RocJpegStreamHandle> hs;
        std::vector<RocJpegImage> imgs;
        for (size_t j = i; j < std::min(items.size(), i + size_t(a.batch)); j++) {
          hs.push_back(items[j].s);
          imgs.push_back(items[j].img);
        }
        const auto t0 = std::chrono::steady_clock::now();
        if (rocJpegDecodeBatched(h, hs.data(), int(hs.size()), &a.params, imgs.data()) != ROCJPEG_STATUS_SUCCESS) {
          fails++;
          break;
        }
        ms += std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
        n += hs.size();
      }
      for (auto &it : items) {
        if (Save(a, is_dir, it)) fails++;
        Free(it);
      }
      if (rocJpegDestroy(h) != ROCJPEG_STATUS_SUCCESS) fails++;
      rate[size_t(t)] = ms > 0 ? 1000.0 * double(n) / ms : 0.0;
    });
  for (auto &x : th) x.join();
  double sum = 0;
  for (double r : rate) sum += r;
  std::printf("threads %d, images/s summed %.1f\n", a.threads, sum);
  return fails.load() ? 1 : 0;
}

}  // namespace

int main(int argc, char **argv) {
  const Args a = Parse(argc, argv);
  if (RJ_SAMPLE_MODE == 2) return RunPerf(a);
  return RunSerial(a, RJ_SAMPLE_MODE == 1);
}
