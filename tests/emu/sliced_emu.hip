// sliced_emu.hip -- host emulation of the bit-sliced GF(2^8) encode
// (csrc/rs_gf8_sliced.hip): the SAME per-lane transform code
// (csrc/leo8_sliced.hpp, compiled for the host), with the kernel's loads, LDS
// layout exchanges and stores replaced by plain loops over the NW waves of a
// workgroup.  Test infrastructure: tests/test_sliced_emu.py compares it with
// the oracle on the CPU, so the algorithm (layouts, skew split, matrices,
// transposes) is checked without a GPU.
#include <stdint.h>
#include <string.h>

#include <vector>

#include "../../celestia-app_amd/csrc/leo8_sliced.hpp"

using namespace dagpu::sliced;

namespace {

template <int K>
void encode_chunk_lane(const uint8_t* data, uint8_t* parity, long shard, long col0) {
  constexpr int NW = Geo<K>::NW;
  static uint32_t st[NW][16][8], tmp[NW][16][8];
  for (int wa = 0; wa < NW; wa++)
    for (int j = 0; j < 16; j++) {
      const uint8_t* src = data + (long)(16 * wa + j) * shard;
      uint32_t d[8];
      memcpy(d, src + col0, 16);
      memcpy(d + 4, src + col0 + 256, 16);
      transpose8(d);
      memcpy(st[wa][j], d, 32);
    }
  for (int wa = 0; wa < NW; wa++) ifft_A<K>(st[wa], &kWMasksHost.m[0][wa][0], kMaxWav * 64);
  for (int wb = 0; wb < NW; wb++)  // A -> B
    for (int i = 0; i < 16; i++) {
      const int e = wb + NW * i;
      memcpy(tmp[wb][i], st[e >> 4][e & 15], 32);
    }
  for (int wb = 0; wb < NW; wb++) {
    ifft_fft_B<K>(tmp[wb]);
  }
  for (int wb = 0; wb < NW; wb++)  // B -> A
    for (int i = 0; i < 16; i++) {
      const int e = wb + NW * i;
      memcpy(st[e >> 4][e & 15], tmp[wb][i], 32);
    }
  for (int wa = 0; wa < NW; wa++) fft_A<K>(st[wa], &kWMasksHost.m[0][wa][0], kMaxWav * 64);
  for (int wa = 0; wa < NW; wa++)
    for (int j = 0; j < 16; j++) {
      uint32_t d[8];
      memcpy(d, st[wa][j], 32);
      transpose8(d);
      uint8_t* dst = parity + (long)(16 * wa + j) * shard;
      memcpy(dst + col0, d, 16);
      memcpy(dst + col0 + 256, d + 4, 16);
    }
}


// Two-vector layout of leo8_encode_sliced2_kernel (k = 128): one vector's
// column block t, the 8 (wave w, lane element bit eb) "lanes" of layout A
// (e = j + 16 eb + 32 w, layer 0), A* (e = eb + 2 r + 32 w, layers 1..2) and
// B (e = eb + 2 w + 8 i).  IO / FO: skew offsets (K / 0 encode, 0 / K reverse fill).
template <int IO, int FO>
void encode2_chunk_lane(const uint8_t* data, uint8_t* parity, long shard, long col0) {
  constexpr int K = 128;
  static uint32_t st[4][2][16][8], tmp[4][2][16][8];
  for (int w = 0; w < 4; w++)
    for (int eb = 0; eb < 2; eb++)
      for (int j = 0; j < 16; j++) {
        const uint8_t* src = data + (long)(j + 16 * eb + 32 * w) * shard;
        uint32_t d[8];
        memcpy(d, src + col0, 16);
        memcpy(d + 4, src + col0 + 256, 16);
        transpose8(d);
        memcpy(st[w][eb][j], d, 32);
      }
  static uint32_t as[4][2][16][8];  // layout A*: e = eb + 2 r + 32 w
  for (int w = 0; w < 4; w++)
    for (int eb = 0; eb < 2; eb++) ifft_A2<K, 1, IO>(st[w][eb], w, eb ? 0xFFFFFFFFu : 0u);
  for (int w = 0; w < 4; w++)  // A -> A* (wave-local)
    for (int eb = 0; eb < 2; eb++)
      for (int r = 0; r < 16; r++) {
        const int e = eb + 2 * r;  // within the wave
        memcpy(as[w][eb][r], st[w][e >> 4][e & 15], 32);
      }
  for (int w = 0; w < 4; w++)
    for (int eb = 0; eb < 2; eb++) ifft_As2<K, IO>(as[w][eb], w);
  for (int w = 0; w < 4; w++)  // A* -> B
    for (int eb = 0; eb < 2; eb++)
      for (int i = 0; i < 16; i++) {
        const int e = eb + 2 * w + 8 * i;
        memcpy(tmp[w][eb][i], as[e >> 5][e & 1][(e >> 1) & 15], 32);
      }
  for (int w = 0; w < 4; w++)
    for (int eb = 0; eb < 2; eb++) {
      ifft_fft_B<K, IO, FO>(tmp[w][eb]);
    }
  for (int w = 0; w < 4; w++)  // B -> A*
    for (int eb = 0; eb < 2; eb++)
      for (int i = 0; i < 16; i++) {
        const int e = eb + 2 * w + 8 * i;
        memcpy(as[e >> 5][e & 1][(e >> 1) & 15], tmp[w][eb][i], 32);
      }
  for (int w = 0; w < 4; w++)
    for (int eb = 0; eb < 2; eb++) fft_As2<K, FO>(as[w][eb], w);
  for (int w = 0; w < 4; w++)  // A* -> A (wave-local)
    for (int eb = 0; eb < 2; eb++)
      for (int r = 0; r < 16; r++) {
        const int e = eb + 2 * r;
        memcpy(st[w][e >> 4][e & 15], as[w][eb][r], 32);
      }
  for (int w = 0; w < 4; w++)
    for (int eb = 0; eb < 2; eb++) fft_A2<K, 1, FO>(st[w][eb], w, eb ? 0xFFFFFFFFu : 0u);
  for (int w = 0; w < 4; w++)
    for (int eb = 0; eb < 2; eb++)
      for (int j = 0; j < 16; j++) {
        uint32_t d[8];
        memcpy(d, st[w][eb][j], 32);
        transpose8(d);
        uint8_t* dst = parity + (long)(j + 16 * eb + 32 * w) * shard;
        memcpy(dst + col0, d, 16);
        memcpy(dst + col0 + 256, d + 4, 16);
      }
}

template <int K>
int encode(long shard, const uint8_t* data, uint8_t* parity) {
  for (long c = 0; c < shard; c += 512)
    for (int t = 0; t < 16; t++) encode_chunk_lane<K>(data, parity, shard, c + 16 * t);
  return 0;
}

}  // namespace

extern "C" int sliced2_emu_encode(long shard, const uint8_t* data, uint8_t* parity) {
  if (shard <= 0 || shard % 512) return -1;
  for (long c = 0; c < shard; c += 512)
    for (int t = 0; t < 16; t++) encode2_chunk_lane<128, 0>(data, parity, shard, c + 16 * t);
  return 0;
}

// reverse fill transform of the k = 128 Repair kernel: 128 parity shards -> data
extern "C" int sliced2_emu_reverse(long shard, const uint8_t* parity, uint8_t* data) {
  if (shard <= 0 || shard % 512) return -1;
  for (long c = 0; c < shard; c += 512)
    for (int t = 0; t < 16; t++) encode2_chunk_lane<0, 128>(parity, data, shard, c + 16 * t);
  return 0;
}

extern "C" int sliced_emu_encode(int k, long shard, const uint8_t* data, uint8_t* parity) {
  if (shard <= 0 || shard % 512) return -1;
  switch (k) {
    case 16: return encode<16>(shard, data, parity);
    case 32: return encode<32>(shard, data, parity);
    case 64: return encode<64>(shard, data, parity);
    case 128: return encode<128>(shard, data, parity);
    default: return -1;
  }
}

// bitop3 emulation and matrices, for a direct unit check
extern "C" uint32_t sliced_emu_bop3(uint32_t a, uint32_t b, uint32_t c, int tt) {
  return sl_bop3_host(a, b, c, (uint8_t)tt);
}
extern "C" int sliced_emu_gmul(int a, int c) { return gmul((uint8_t)a, (uint8_t)c); }

// ---------------------------------------------------------------------------
// Bit-sliced k = 128 decode (csrc/rs_decode_sliced.hip): the kernel's error
// locators (leo8_errlocs_kernel), premultiply, dec_A / dec_B, formal
// derivative and postmultiply, with the 16 (wave w, lane group eb) lanes of a
// column block as loops and the LDS passes as copies.
// ---------------------------------------------------------------------------
namespace {

uint32_t add_mod8(uint32_t a, uint32_t b) { const uint32_t s = a + b; return (s + (s >> 8)) & 0xFFu; }
uint32_t sub_mod8(uint32_t a, uint32_t b) { const uint32_t d = a - b; return (d + (d >> 8)) & 0xFFu; }

void fwht256(uint32_t* e, int mtrunc) {
  for (int dist = 1; dist <= 64; dist *= 4) {
    const int dist4 = dist * 4;
    for (int g = 0; g < 64; g++) {
      const int r = (g / dist) * dist4;
      const int i = r + (g % dist);
      if (r >= mtrunc) continue;
      const uint32_t t0 = e[i], t1 = e[i + dist], t2 = e[i + 2 * dist], t3 = e[i + 3 * dist];
      const uint32_t a0 = add_mod8(t0, t1), a1 = sub_mod8(t0, t1);
      const uint32_t a2 = add_mod8(t2, t3), a3 = sub_mod8(t2, t3);
      e[i] = add_mod8(a0, a2);
      e[i + 2 * dist] = sub_mod8(a0, a2);
      e[i + dist] = add_mod8(a1, a3);
      e[i + 3 * dist] = sub_mod8(a1, a3);
    }
  }
}

int elemA(int r, int eb, int w) { return r + 16 * eb + 64 * w; }
int elemS(int r, int eb, int w) { return eb + 4 * r + 64 * w; }  // A*
int elemB(int r, int eb, int w) { return eb + 4 * w + 16 * r; }

// wave-local A <-> A* (the kernel's dec_transpose_wave): per wave, element
// e = j + 16 eb moves to lane group e & 3, register e >> 2
void a_to_s(uint32_t (&st)[4][4][16][8], bool forward) {
  static uint32_t tmp[4][4][16][8];
  for (int w = 0; w < 4; w++)
    for (int eb = 0; eb < 4; eb++)
      for (int r = 0; r < 16; r++) {
        const int e = forward ? elemS(r, eb, 0) : elemA(r, eb, 0);  // destination element
        const int src_eb = forward ? (e >> 4) : (e & 3), src_r = forward ? (e & 15) : (e >> 2);
        memcpy(tmp[w][eb][r], st[w][src_eb][src_r], 32);
      }
  memcpy(st, tmp, sizeof(tmp));
}

}  // namespace

// shards: 256 x shard bytes, [data 128][parity 128] (shard order), repaired in
// place; present: 256 flags in shard order.  Returns -1 on bad arguments.
extern "C" int sliced_dec_emu(long shard, uint8_t* shards, const uint8_t* present) {
  constexpr int K = 128, N = 256;
  if (shard <= 0 || shard % 512) return -1;
  auto shard_of = [&](int e) { return e < K ? e + K : e - K; };  // work index -> shard
  uint32_t err[N];
  for (int i = 0; i < N; i++) err[i] = present[shard_of(i)] ? 0u : 1u;
  fwht256(err, N);
  for (int i = 0; i < N; i++) err[i] = (err[i] * dagpu::kGf8.walsh[i]) % 255u;
  fwht256(err, N);
  static uint32_t st[4][4][16][8], tmp[4][4][16][8], orig[4][4][16][8];
  for (long c = 0; c < shard; c += 512)
    for (int t = 0; t < 16; t++) {
      const long col0 = c + 16 * t;
      for (int w = 0; w < 4; w++)
        for (int eb = 0; eb < 4; eb++)
          for (int j = 0; j < 16; j++) {
            const int e = elemA(j, eb, w);
            const uint8_t* src = shards + (long)shard_of(e) * shard;
            uint32_t d[8];
            memcpy(d, src + col0, 16);
            memcpy(d + 4, src + col0 + 256, 16);
            const int lm = present[shard_of(e)] ? (int)(err[e] & 0xFF) : -1;
            mul_packed(d, mul_table(lm), mul_table2(lm));
            transpose8(d);
            memcpy(st[w][eb][j], d, 32);
          }
      for (int w = 0; w < 4; w++)
        for (int eb = 0; eb < 4; eb++)
          dec_A<true, 2>(st[w][eb], w, (eb & 1) ? 0xFFFFFFFFu : 0u, (eb & 2) ? 0xFFFFFFFFu : 0u);
      a_to_s(st, true);
      for (int w = 0; w < 4; w++)
        for (int eb = 0; eb < 4; eb++) dec_Astar<true>(st[w][eb], w);
      for (int w = 0; w < 4; w++)  // A* -> B
        for (int eb = 0; eb < 4; eb++)
          for (int i = 0; i < 16; i++) {
            const int e = elemB(i, eb, w);  // held in A* by wave e >> 6, lane group e & 3, register (e >> 2) & 15
            memcpy(tmp[w][eb][i], st[e >> 6][e & 3][(e >> 2) & 15], 32);
          }
      for (int w = 0; w < 4; w++)
        for (int eb = 0; eb < 4; eb++) dec_B<true>(tmp[w][eb]);
      memcpy(orig, tmp, sizeof(orig));
      for (int w = 0; w < 4; w++)
        for (int eb = 0; eb < 4; eb++) {
          deriv_local<0, 8>(tmp[w][eb]);
          for (int i = 0; i < 16; i++) {
            const int e = elemB(i, eb, w);
            for (int s = 0; s < 4; s++) {
              if ((e >> s) & 1) continue;
              const int f = e | (1 << s);  // partner in layout B: eb' = f & 3, w' = (f >> 2) & 3, i' = f >> 4
              for (int p = 0; p < 8; p++) tmp[w][eb][i][p] ^= orig[(f >> 2) & 3][f & 3][f >> 4][p];
            }
          }
        }
      for (int w = 0; w < 4; w++)
        for (int eb = 0; eb < 4; eb++) dec_B<false>(tmp[w][eb]);
      for (int w = 0; w < 4; w++)  // B -> A*
        for (int eb = 0; eb < 4; eb++)
          for (int i = 0; i < 16; i++) {
            const int e = elemB(i, eb, w);
            memcpy(st[e >> 6][e & 3][(e >> 2) & 15], tmp[w][eb][i], 32);
          }
      for (int w = 0; w < 4; w++)
        for (int eb = 0; eb < 4; eb++) dec_Astar<false>(st[w][eb], w);
      a_to_s(st, false);
      for (int w = 0; w < 4; w++)
        for (int eb = 0; eb < 4; eb++)
          dec_A<false, 2>(st[w][eb], w, (eb & 1) ? 0xFFFFFFFFu : 0u, (eb & 2) ? 0xFFFFFFFFu : 0u);
      for (int w = 0; w < 4; w++)
        for (int eb = 0; eb < 4; eb++)
          for (int j = 0; j < 16; j++) {
            const int e = elemA(j, eb, w);
            if (present[shard_of(e)]) continue;
            uint32_t d[8];
            memcpy(d, st[w][eb][j], 32);
            transpose8(d);
            const int lm = (int)(255u - (err[e] & 0xFF));
            mul_packed(d, mul_table(lm), mul_table2(lm));
            uint8_t* dst = shards + (long)shard_of(e) * shard;
            memcpy(dst + col0, d, 16);
            memcpy(dst + col0 + 256, d + 4, 16);
          }
    }
  return 0;
}
