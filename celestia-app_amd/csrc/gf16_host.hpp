// gf16_host.hpp -- host generation of the Leopard GF(2^16) tables
// (klauspost/reedsolomon v1.11.8 leopard.go initLUTs / initFFTSkew), uploaded
// once per context for the GF(2^16) kernels (rs_gf16.hip).  Product code: the
// tables are constants of the codec, like the constexpr GF(2^8) ones.
#pragma once
#include <stdint.h>

#include <vector>

namespace dagpu {
namespace gf16 {

constexpr int kBits = 16;
constexpr int kOrder = 65536;
constexpr int kMod = 65535;

inline uint16_t add_mod(unsigned a, unsigned b) {
  unsigned s = a + b;
  return (uint16_t)(s + (s >> kBits));
}
inline uint16_t sub_mod(unsigned a, unsigned b) {
  uint64_t d = (uint64_t)a - (uint64_t)b;
  return (uint16_t)(d + (d >> kBits));
}

struct Tables {
  std::vector<uint16_t> log, exp, skew, walsh;
};

inline void fwht(uint16_t* data, int m, int mtrunc) {
  int dist = 1, dist4 = 4;
  while (dist4 <= m) {
    for (int r = 0; r < mtrunc; r += dist4) {
      for (int i = r; i < r + dist; i++) {
        uint16_t t0 = data[i], t1 = data[i + dist], t2 = data[i + 2 * dist], t3 = data[i + 3 * dist];
        uint16_t a0 = add_mod(t0, t1), a1 = sub_mod(t0, t1), a2 = add_mod(t2, t3), a3 = sub_mod(t2, t3);
        data[i] = add_mod(a0, a2); data[i + 2 * dist] = sub_mod(a0, a2);
        data[i + dist] = add_mod(a1, a3); data[i + 3 * dist] = sub_mod(a1, a3);
      }
    }
    dist = dist4;
    dist4 <<= 2;
  }
  if (dist < m) {
    for (int i = 0; i < dist; i++) {
      uint16_t a = data[i], b = data[i + dist];
      data[i] = add_mod(a, b);
      data[i + dist] = sub_mod(a, b);
    }
  }
}

inline Tables make_tables() {
  static const uint16_t cantor[16] = {0x0001, 0xACCA, 0x3C0E, 0x163E, 0xC582, 0xED2E, 0x914C, 0x4012,
                                      0x6C98, 0x10D8, 0x6A72, 0xB900, 0xFDB8, 0xFB34, 0xFF38, 0x991E};
  Tables t;
  t.log.assign(kOrder, 0);
  t.exp.assign(kOrder, 0);
  t.skew.assign(kOrder, 0);  // kMod used entries (+1 pad)
  t.walsh.assign(kOrder, 0);
  unsigned state = 1;
  for (unsigned i = 0; i < (unsigned)kMod; i++) {
    t.exp[state] = (uint16_t)i;
    state <<= 1;
    if (state >= (unsigned)kOrder) state ^= 0x1002D;
  }
  t.exp[0] = kMod;
  t.log[0] = 0;
  for (int i = 0; i < kBits; i++) {
    int width = 1 << i;
    for (int j = 0; j < width; j++) t.log[j + width] = t.log[j] ^ cantor[i];
  }
  for (int i = 0; i < kOrder; i++) t.log[i] = t.exp[t.log[i]];
  for (int i = 0; i < kOrder; i++) t.exp[t.log[i]] = (uint16_t)i;
  t.exp[kMod] = t.exp[0];
  auto mullog = [&](uint16_t a, uint16_t lb) -> uint16_t {
    if (a == 0) return 0;
    return t.exp[add_mod(t.log[a], lb)];
  };
  uint16_t temp[kBits - 1];
  for (int i = 1; i < kBits; i++) temp[i - 1] = (uint16_t)(1 << i);
  for (int m = 0; m < kBits - 1; m++) {
    int step = 1 << (m + 1);
    t.skew[(1 << m) - 1] = 0;
    for (int i = m; i < kBits - 1; i++) {
      int s = 1 << (i + 1);
      for (int j = (1 << m) - 1; j < s; j += step) t.skew[j + s] = t.skew[j] ^ temp[i];
    }
    temp[m] = (uint16_t)(kMod - t.log[mullog(temp[m], t.log[temp[m] ^ 1])]);
    for (int i = m + 1; i < kBits - 1; i++) {
      uint16_t sum = add_mod(t.log[temp[i] ^ 1], temp[m]);
      temp[i] = mullog(temp[i], sum);
    }
  }
  for (int i = 0; i < kMod; i++) t.skew[i] = t.log[t.skew[i]];
  for (int i = 0; i < kOrder; i++) t.walsh[i] = t.log[i];
  t.walsh[0] = 0;
  fwht(t.walsh.data(), kOrder, kOrder);
  return t;
}

}  // namespace gf16
}  // namespace dagpu
