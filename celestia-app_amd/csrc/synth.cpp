// synth.cpp -- fast seeded generator of the benchmark input (libdasynth.so).
//
// Bench/test infrastructure, not part of the DA path: block replay (configs[4])
// needs thousands of DISTINCT 128x128 squares in host memory, which the numpy
// generator (celestia_da/synth.py random_blob_square) produces at ~30 ms per
// square.  Same shape of data: "random-namespace blob shares"
// (test/util/testfactory/common.go:36-46): 512 random bytes per share, bytes
// [0:29] = blob namespace version 0 | 18 zero bytes | 10 random bytes, not
// reserved (pkg/namespace/random_blob.go:22-30: an ID whose first 9 random
// bytes are zero is reserved, fixed by setting the first to 1 as synth.py
// does), then all k^2 shares sorted bytewise so every Q0 row and column is in
// NMT push order.  The PRNG is a counter-based SplitMix64 stream per square
// (square index i of a run seeded `seed` is the same bytes whatever `first`
// and `count` select), so any block can be regenerated on its own for checks.
#include <stdint.h>
#include <string.h>

#include <algorithm>
#include <thread>
#include <vector>

namespace {

constexpr size_t kShare = 512;

inline uint64_t mix64(uint64_t z) {
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

// Share o of a square is the 64 SplitMix64 words o*64 .. o*64+63 of the
// square's stream (little-endian), with bytes [0:19) zeroed and the reserved
// fix applied.  Only the namespace keys are sorted; each share's bytes are
// then generated straight into its sorted slot (no staging copy).
struct Key {
  uint64_t hi;  // namespace bytes 19..26, big-endian (compares like bytes)
  uint32_t lo;  // bytes 27..28
  uint32_t o;   // original share index
};

inline void gen_share(uint64_t base, uint64_t o, uint8_t* dst) {
  uint64_t* w = reinterpret_cast<uint64_t*>(dst);
  for (uint64_t j = 0; j < 64; j++) w[j] = mix64(base + (o * 64 + j) * 0x9E3779B97F4A7C15ull);
  bool zero9 = true;
  for (int b = 19; b < 28; b++) zero9 &= dst[b] == 0;
  memset(dst, 0, 19);  // version 0 + NamespaceVersionZeroPrefix
  if (zero9) dst[19] = 1;  // reserved ID -> blob ID
}

inline Key key_of(uint64_t base, uint32_t o) {
  uint8_t ns[32];
  uint64_t* w = reinterpret_cast<uint64_t*>(ns);
  for (uint64_t j = 2; j < 4; j++) w[j] = mix64(base + ((uint64_t)o * 64 + j) * 0x9E3779B97F4A7C15ull);
  bool zero9 = true;
  for (int b = 19; b < 28; b++) zero9 &= ns[b] == 0;
  if (zero9) ns[19] = 1;
  Key key{0, 0, o};
  for (int b = 19; b < 27; b++) key.hi = (key.hi << 8) | ns[b];
  key.lo = ((uint32_t)ns[27] << 8) | ns[28];
  return key;
}

void one_square(uint32_t k, uint64_t seed, uint64_t index, uint8_t* out, std::vector<Key>& keys) {
  const size_t n = (size_t)k * k;
  const uint64_t base = mix64(seed * 0x9E3779B97F4A7C15ull + mix64(index + 0x632BE59BD9B4E019ull));
  keys.resize(n);
  for (size_t s = 0; s < n; s++) keys[s] = key_of(base, (uint32_t)s);
  std::sort(keys.begin(), keys.end(), [](const Key& a, const Key& b) {
    return a.hi != b.hi ? a.hi < b.hi : a.lo != b.lo ? a.lo < b.lo : a.o < b.o;
  });
  for (size_t s = 0; s < n; s++) gen_share(base, keys[s].o, out + s * kShare);
  // equal namespaces (probability ~n^2 / 2^81): order that run by full bytes
  for (size_t s = 0; s + 1 < n;) {
    size_t e = s + 1;
    while (e < n && keys[e].hi == keys[s].hi && keys[e].lo == keys[s].lo) e++;
    if (e - s > 1) {
      std::vector<uint8_t> run((e - s) * kShare);
      memcpy(run.data(), out + s * kShare, run.size());
      std::vector<size_t> idx(e - s);
      for (size_t i = 0; i < idx.size(); i++) idx[i] = i;
      std::sort(idx.begin(), idx.end(), [&](size_t a, size_t b) {
        return memcmp(run.data() + a * kShare, run.data() + b * kShare, kShare) < 0;
      });
      for (size_t i = 0; i < idx.size(); i++)
        memcpy(out + (s + i) * kShare, run.data() + idx[i] * kShare, kShare);
    }
    s = e;
  }
}

}  // namespace

extern "C" {

// Squares first .. first+count-1 of the run `seed`, each k*k*512 bytes, packed
// into `out`.  nthreads <= 0: one per hardware thread.  Returns 0, or -1 on a
// bad argument.
int dasynth_blob_squares(uint32_t k, uint64_t seed, uint64_t first, uint64_t count, uint8_t* out,
                         int nthreads) {
  if (k == 0 || (count && !out)) return -1;
  if (nthreads <= 0) nthreads = (int)std::max(1u, std::thread::hardware_concurrency());
  if ((uint64_t)nthreads > count) nthreads = (int)std::max<uint64_t>(1, count);
  const size_t sq = (size_t)k * k * kShare;
  auto work = [&](int t) {
    std::vector<Key> keys;
    for (uint64_t i = (uint64_t)t; i < count; i += (uint64_t)nthreads)
      one_square(k, seed, first + i, out + i * sq, keys);
  };
  if (nthreads == 1) {
    work(0);
    return 0;
  }
  std::vector<std::thread> pool;
  for (int t = 0; t < nthreads; t++) pool.emplace_back(work, t);
  for (auto& th : pool) th.join();
  return 0;
}

}  // extern "C"
