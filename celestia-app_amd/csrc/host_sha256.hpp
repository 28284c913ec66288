// host_sha256.hpp -- host-side SHA-256 and RFC-6962 root for the small,
// off-hot-path hashes of the boundary: DataAvailabilityHeader.Hash() on roots a
// caller already holds (e.g. a DAH decoded from its proto form,
// pkg/da/data_availability_header.go:92-108, 122-132) and the nil-DAH case.
// The hot path computes the DAH on the GPU (nmt.hip dah_kernel).
#pragma once
#include <stddef.h>
#include <stdint.h>
#include <string.h>

#include <vector>

namespace dagpu {
namespace host {

struct Sha256 {
  uint32_t h[8];
  uint8_t buf[64];
  size_t nbuf = 0;
  uint64_t len = 0;
  Sha256() {
    static const uint32_t iv[8] = {0x6a09e667, 0xbb67ae85, 0x3c6ef372, 0xa54ff53a,
                                   0x510e527f, 0x9b05688c, 0x1f83d9ab, 0x5be0cd19};
    memcpy(h, iv, sizeof h);
  }
  static uint32_t ror(uint32_t x, int n) { return (x >> n) | (x << (32 - n)); }
  void block(const uint8_t* p) {
    static const uint32_t K[64] = {
        0x428a2f98, 0x71374491, 0xb5c0fbcf, 0xe9b5dba5, 0x3956c25b, 0x59f111f1, 0x923f82a4,
        0xab1c5ed5, 0xd807aa98, 0x12835b01, 0x243185be, 0x550c7dc3, 0x72be5d74, 0x80deb1fe,
        0x9bdc06a7, 0xc19bf174, 0xe49b69c1, 0xefbe4786, 0x0fc19dc6, 0x240ca1cc, 0x2de92c6f,
        0x4a7484aa, 0x5cb0a9dc, 0x76f988da, 0x983e5152, 0xa831c66d, 0xb00327c8, 0xbf597fc7,
        0xc6e00bf3, 0xd5a79147, 0x06ca6351, 0x14292967, 0x27b70a85, 0x2e1b2138, 0x4d2c6dfc,
        0x53380d13, 0x650a7354, 0x766a0abb, 0x81c2c92e, 0x92722c85, 0xa2bfe8a1, 0xa81a664b,
        0xc24b8b70, 0xc76c51a3, 0xd192e819, 0xd6990624, 0xf40e3585, 0x106aa070, 0x19a4c116,
        0x1e376c08, 0x2748774c, 0x34b0bcb5, 0x391c0cb3, 0x4ed8aa4a, 0x5b9cca4f, 0x682e6ff3,
        0x748f82ee, 0x78a5636f, 0x84c87814, 0x8cc70208, 0x90befffa, 0xa4506ceb, 0xbef9a3f7,
        0xc67178f2};
    uint32_t w[64];
    for (int i = 0; i < 16; i++)
      w[i] = ((uint32_t)p[4 * i] << 24) | ((uint32_t)p[4 * i + 1] << 16) |
             ((uint32_t)p[4 * i + 2] << 8) | p[4 * i + 3];
    for (int i = 16; i < 64; i++) {
      uint32_t s0 = ror(w[i - 15], 7) ^ ror(w[i - 15], 18) ^ (w[i - 15] >> 3);
      uint32_t s1 = ror(w[i - 2], 17) ^ ror(w[i - 2], 19) ^ (w[i - 2] >> 10);
      w[i] = w[i - 16] + s0 + w[i - 7] + s1;
    }
    uint32_t a = h[0], b = h[1], c = h[2], d = h[3], e = h[4], f = h[5], g = h[6], hh = h[7];
    for (int i = 0; i < 64; i++) {
      uint32_t t1 = hh + (ror(e, 6) ^ ror(e, 11) ^ ror(e, 25)) + ((e & f) ^ (~e & g)) + K[i] + w[i];
      uint32_t t2 = (ror(a, 2) ^ ror(a, 13) ^ ror(a, 22)) + ((a & b) ^ (a & c) ^ (b & c));
      hh = g; g = f; f = e; e = d + t1; d = c; c = b; b = a; a = t1 + t2;
    }
    h[0] += a; h[1] += b; h[2] += c; h[3] += d; h[4] += e; h[5] += f; h[6] += g; h[7] += hh;
  }
  void update(const uint8_t* p, size_t n) {
    len += n;
    while (n) {
      size_t t = 64 - nbuf < n ? 64 - nbuf : n;
      memcpy(buf + nbuf, p, t);
      nbuf += t; p += t; n -= t;
      if (nbuf == 64) { block(buf); nbuf = 0; }
    }
  }
  void final(uint8_t out[32]) {
    uint64_t bits = len * 8;
    uint8_t pad = 0x80;
    update(&pad, 1);
    uint8_t z = 0;
    while (nbuf != 56) update(&z, 1);
    uint8_t lb[8];
    for (int i = 0; i < 8; i++) lb[i] = (uint8_t)(bits >> (56 - 8 * i));
    update(lb, 8);
    for (int i = 0; i < 8; i++) {
      out[4 * i] = h[i] >> 24; out[4 * i + 1] = h[i] >> 16;
      out[4 * i + 2] = h[i] >> 8; out[4 * i + 3] = h[i];
    }
  }
};

inline void rfc6962_rec(const std::vector<const uint8_t*>& items, size_t lo, size_t hi,
                        size_t len, uint8_t out[32]) {
  const size_t n = hi - lo;
  if (n == 1) {
    Sha256 s;
    uint8_t z = 0x00;
    s.update(&z, 1);
    s.update(items[lo], len);
    s.final(out);
    return;
  }
  size_t split = 1;
  while (split * 2 < n) split *= 2;
  uint8_t l[32], r[32];
  rfc6962_rec(items, lo, lo + split, len, l);
  rfc6962_rec(items, lo + split, hi, len, r);
  Sha256 s;
  uint8_t one = 0x01;
  s.update(&one, 1);
  s.update(l, 32);
  s.update(r, 32);
  s.final(out);
}

// celestia-core crypto/merkle HashFromByteSlices: empty -> SHA256("").
inline void rfc6962_root(const std::vector<const uint8_t*>& items, size_t len, uint8_t out[32]) {
  if (items.empty()) {
    Sha256 s;
    s.final(out);
    return;
  }
  rfc6962_rec(items, 0, items.size(), len, out);
}

// ---- proof verification (off the hot path: a light client checks a few nodes) ----

constexpr size_t kNs = 29, kNodeLen = 90;

// nmt HashLeaf (test/util/malicious/hasher.go:186-212 mirror of nmt v0.20.0):
// ns || ns || SHA256(0x00 || ns || data)
inline void nmt_hash_leaf(const uint8_t* ns, const uint8_t* data, size_t len, uint8_t out[kNodeLen]) {
  uint8_t tmp[kNodeLen];
  memcpy(tmp, ns, kNs);
  memcpy(tmp + kNs, ns, kNs);
  Sha256 s;
  const uint8_t z = 0x00;
  s.update(&z, 1);
  s.update(ns, kNs);
  s.update(data, len);
  s.final(tmp + 2 * kNs);
  memcpy(out, tmp, kNodeLen);
}

// nmt HashNode with IgnoreMaxNamespace (hasher.go:271-309): false when the
// siblings are unordered (right.min < left.max, nmt ErrUnorderedSiblings).
inline bool nmt_hash_node(const uint8_t* l, const uint8_t* r, uint8_t out[kNodeLen]) {
  if (memcmp(r, l + kNs, kNs) < 0) return false;
  bool rpar = true;
  for (size_t i = 0; i < kNs; i++) rpar &= r[i] == 0xFF;
  uint8_t tmp[kNodeLen];
  memcpy(tmp, l, kNs);
  memcpy(tmp + kNs, rpar ? l + kNs : r + kNs, kNs);
  Sha256 s;
  const uint8_t one = 0x01;
  s.update(&one, 1);
  s.update(l, kNodeLen);
  s.update(r, kNodeLen);
  s.final(tmp + 2 * kNs);
  memcpy(out, tmp, kNodeLen);
  return true;
}

inline void merkle_leaf_hash(const uint8_t* leaf, size_t len, uint8_t out[32]) {
  Sha256 s;
  const uint8_t z = 0x00;
  s.update(&z, 1);
  s.update(leaf, len);
  s.final(out);
}

inline void merkle_inner_hash(const uint8_t* l, const uint8_t* r, uint8_t out[32]) {
  Sha256 s;
  const uint8_t one = 0x01;
  s.update(&one, 1);
  s.update(l, 32);
  s.update(r, 32);
  s.final(out);
}

}  // namespace host
}  // namespace dagpu
