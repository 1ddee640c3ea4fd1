// Driver of the coalescing stub test: T threads, a handle each, batch-1 calls (every 7th call of
// thread 0 a bad stream); checks every call's own status and prints the counters.
#include <cstdio>
#include <cstdlib>
#include <thread>
#include <vector>

#include "rj_coalesce.h"
#include "rj_decoder.h"

int main(int argc, char **argv) {
  const int T = argc > 1 ? std::atoi(argv[1]) : 8, calls = argc > 2 ? std::atoi(argv[2]) : 1000;
  std::vector<rj::Decoder> decs(T);
  std::vector<std::thread> th;
  std::vector<int> wrong(T, 0), nbad(T, 0);
  for (int t = 0; t < T; t++)
    th.emplace_back([&, t] {
      rj::Stream st;
      st.owner = t;
      rj::Stream *sp = &st;
      RocJpegDecodeParams p{};
      p.output_format = (t % 3 == 2) ? ROCJPEG_OUTPUT_RGB : ROCJPEG_OUTPUT_NATIVE;  // two parameter sets
      RocJpegImage img{};
      img.pitch[0] = uint32_t(t);
      for (int i = 0; i < calls; i++) {
        st.bad = t == 0 && i % 7 == 3;
        nbad[t] += st.bad ? 1 : 0;
        const int r = rj::CoalescedDecode(&decs[t], 0, &sp, 1, &p, &img);
        if (r != (st.bad ? ROCJPEG_STATUS_BAD_JPEG : 0)) wrong[t]++;
      }
    });
  for (auto &x : th) x.join();
  long img = 0, att = 0;
  for (auto &d : decs) {
    img += d.images;
    att += d.attempts;
  }
  int bad = 0, bad_calls = 0;
  for (int w : wrong) bad += w;
  for (int b : nbad) bad_calls += b;
  uint64_t a, b, c;
  rj::CoalesceStats(&a, &b, &c);
  std::printf("calls %llu combined %llu members %llu images %ld wrong_status %d bad_calls %d attempts %ld\n", (unsigned long long)a,
              (unsigned long long)b, (unsigned long long)c, img, bad, bad_calls, att);
  return bad ? 1 : 0;
}
