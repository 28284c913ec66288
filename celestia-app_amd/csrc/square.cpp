// square.cpp -- original data square construction on the host side of the C
// ABI: the txs -> ODS step of block replay, before the GPU
// extends the square (app/extend_block.go:14-22: square.Construct then
// da.ExtendShares).  Byte bookkeeping, no device code.
//
// Restates, for app version 1 (SquareSizeUpperBound 128, SubtreeRootThreshold 64):
//   square.Construct / square.Build         pkg/square/square.go:22-63
//   Builder (AppendTx, AppendBlobTx, Export) pkg/square/builder.go
//   WriteSquare                             pkg/square/square.go
//   CompactShareCounter                     pkg/shares/counter.go
//   CompactShareSplitter                    pkg/shares/split_compact_shares.go
//   SparseShareSplitter                     pkg/shares/split_sparse_shares.go
//   Builder (share)                         pkg/shares/share_builder.go
//   padding shares                          pkg/shares/padding.go
//   blob.UnmarshalBlobTx                    pkg/blob/blob.go:56-90 (gogoproto wire format)
//   IndexWrapper marshal                    celestia-core proto/tendermint/types (type_id "INDX")
//   inclusion.SubTreeWidth / NextShareIndex pkg/inclusion/blob_share_commitment_rules.go
// with the error texts of the Python mirror (celestia_da/square.py,
// shares.py), which tests/test_square_native.py compares byte for byte.
// Shares are written straight into the caller's ODS buffer: no per-share
// allocation (the Python mirror takes ~0.17 s per full 128 x 128 square).
#include <stdint.h>
#include <string.h>

#include <algorithm>
#include <cmath>
#include <string>
#include <vector>

#include "../../include/dagpu.h"
#include "runtime.hpp"

namespace {

constexpr size_t kShare = 512, kNs = 29, kNsId = 28;
constexpr size_t kFirstCompact = 474, kContCompact = 478;  // content bytes
constexpr size_t kFirstSparse = 478, kContSparse = 482;

struct SquareError {
  std::string msg;
};

// ---- namespaces (pkg/namespace/consts.go) ----------------------------------
struct Ns {
  uint8_t b[kNs];
};
Ns primary_reserved(uint8_t last) {
  Ns n{};
  n.b[kNs - 1] = last;
  return n;
}
Ns secondary_reserved(uint8_t last) {
  Ns n;
  memset(n.b, 0xFF, kNs);
  n.b[kNs - 1] = last;
  return n;
}
const Ns kTxNs = primary_reserved(0x01);
const Ns kPfbNs = primary_reserved(0x04);
const Ns kReservedPaddingNs = primary_reserved(0xFF);
const Ns kTailPaddingNs = secondary_reserved(0xFE);

// namespace.From: version 0 or 255; a version-0 ID starts with 18 zero bytes
void validate_namespace(const uint8_t* ns) {
  const uint8_t v = ns[0];
  if (v != 0 && v != 255) throw SquareError{"unsupported namespace version " + std::to_string(v)};
  if (v == 0)
    for (int i = 1; i <= 18; i++)
      if (ns[i])
        throw SquareError{"unsupported namespace id with version 0. ID must start with 18 leading zeros"};
}

// ---- varints / proto wire format ---------------------------------------------
size_t uvarint_len(uint64_t v) {
  size_t n = 1;
  while (v >= 0x80) {
    v >>= 7;
    n++;
  }
  return n;
}
size_t put_uvarint(uint8_t* out, uint64_t v) {
  size_t n = 0;
  while (v >= 0x80) {
    out[n++] = (uint8_t)(v | 0x80);
    v >>= 7;
  }
  out[n++] = (uint8_t)v;
  return n;
}
void append_uvarint(std::vector<uint8_t>& o, uint64_t v) {
  uint8_t b[10];
  o.insert(o.end(), b, b + put_uvarint(b, v));
}

struct Span {
  const uint8_t* p = nullptr;
  size_t n = 0;
};

bool read_varint(const uint8_t* b, size_t n, size_t& i, uint64_t& v) {
  v = 0;
  for (unsigned s = 0;; s += 7) {
    if (i >= n || s >= 64) return false;  // unexpected EOF / integer overflow
    const uint8_t c = b[i++];
    v |= (uint64_t)(c & 0x7F) << s;
    if (c < 0x80) return true;
  }
}

// gogoproto-style field walk: calls f(num, wire type, varint, bytes); false on
// a malformed buffer or when f rejects a field (wrong wire type).
template <class F>
bool walk_fields(Span buf, F&& f) {
  size_t i = 0;
  while (i < buf.n) {
    uint64_t key, v = 0;
    if (!read_varint(buf.p, buf.n, i, key)) return false;
    const uint64_t num = key >> 3;
    const int wt = (int)(key & 7);
    if (num == 0) return false;
    Span bytes;
    switch (wt) {
      case 0:
        if (!read_varint(buf.p, buf.n, i, v)) return false;
        break;
      case 1:
        if (i + 8 > buf.n) return false;
        i += 8;
        break;
      case 2: {
        uint64_t len;
        if (!read_varint(buf.p, buf.n, i, len) || len > buf.n - i) return false;
        bytes = {buf.p + i, (size_t)len};
        i += (size_t)len;
        break;
      }
      case 5:
        if (i + 4 > buf.n) return false;
        i += 4;
        break;
      default:
        return false;
    }
    if (!f(num, wt, v, bytes)) return false;
  }
  return true;
}

struct BlobRef {
  Span ns_id, data;
  uint32_t share_version = 0, ns_version = 0;
};

// blob.UnmarshalBlobTx: is a blob tx iff it decodes, type_id == "BLOB", it
// carries blobs and every namespace ID is 28 bytes
bool unmarshal_blob_tx(Span buf, Span& inner, std::vector<BlobRef>& blobs) {
  blobs.clear();
  inner = {};
  Span type_id;
  const bool ok = walk_fields(buf, [&](uint64_t num, int wt, uint64_t, Span b) {
    if (num == 1) {
      if (wt != 2) return false;
      inner = b;
    } else if (num == 2) {
      if (wt != 2) return false;
      BlobRef r;
      const bool ok2 = walk_fields(b, [&](uint64_t n2, int w2, uint64_t v2, Span b2) {
        if (n2 == 1) {
          if (w2 != 2) return false;
          r.ns_id = b2;
        } else if (n2 == 2) {
          if (w2 != 2) return false;
          r.data = b2;
        } else if (n2 == 3) {
          if (w2 != 0) return false;
          r.share_version = (uint32_t)v2;
        } else if (n2 == 4) {
          if (w2 != 0) return false;
          r.ns_version = (uint32_t)v2;
        }
        return true;
      });
      if (!ok2) return false;
      blobs.push_back(r);
    } else if (num == 3) {
      if (wt != 2) return false;
      type_id = b;
    }
    return true;
  });
  if (!ok) return false;
  if (type_id.n != 4 || memcmp(type_id.p, "BLOB", 4) != 0 || blobs.empty()) return false;
  for (const auto& b : blobs)
    if (b.ns_id.n != kNsId) return false;
  return true;
}

// tmproto.IndexWrapper{tx = 1, share_indexes = 2 (packed), type_id = 3 "INDX"}
void marshal_index_wrapper(Span tx, const std::vector<uint32_t>& idx, std::vector<uint8_t>& o) {
  o.clear();
  if (tx.n) {
    o.push_back(0x0a);
    append_uvarint(o, tx.n);
    o.insert(o.end(), tx.p, tx.p + tx.n);
  }
  if (!idx.empty()) {
    size_t packed = 0;
    for (uint32_t x : idx) packed += uvarint_len(x);
    o.push_back(0x12);
    append_uvarint(o, packed);
    for (uint32_t x : idx) append_uvarint(o, x);
  }
  o.push_back(0x1a);
  o.push_back(4);
  o.insert(o.end(), {'I', 'N', 'D', 'X'});
}
size_t index_wrapper_size(size_t tx_len, size_t n_idx, uint32_t each) {
  size_t s = 6;  // type_id field
  if (tx_len) s += 1 + uvarint_len(tx_len) + tx_len;
  if (n_idx) {
    const size_t packed = n_idx * uvarint_len(each);
    s += 1 + uvarint_len(packed) + packed;
  }
  return s;
}

// ---- shares ---------------------------------------------------------------------
uint64_t round_up_pow2(uint64_t v) {
  uint64_t r = 1;
  while (r < v) r <<= 1;
  return r;
}
uint64_t blob_min_square_size(uint64_t share_count) {
  return round_up_pow2((uint64_t)std::ceil(std::sqrt((double)share_count)));
}
uint64_t subtree_width_u(uint64_t share_count, uint64_t threshold) {
  uint64_t s = share_count / threshold + (share_count % threshold ? 1 : 0);
  s = round_up_pow2(s);
  const uint64_t m = blob_min_square_size(share_count);
  return s < m ? s : m;
}
uint64_t sparse_shares_needed(uint64_t len) {
  if (len == 0) return 0;
  if (len < kFirstSparse) return 1;
  return 1 + (len - kFirstSparse + kContSparse - 1) / kContSparse;
}
void put_be32(uint8_t* p, uint32_t v) {
  p[0] = (uint8_t)(v >> 24);
  p[1] = (uint8_t)(v >> 16);
  p[2] = (uint8_t)(v >> 8);
  p[3] = (uint8_t)v;
}
uint32_t get_be32(const uint8_t* p) { return (uint32_t)p[0] << 24 | (uint32_t)p[1] << 16 | (uint32_t)p[2] << 8 | p[3]; }

// namespace padding share: ns | info(version, start) | sequence len 0 | zeros
void padding_share(uint8_t* out, const uint8_t* ns, uint8_t version) {
  memcpy(out, ns, kNs);
  out[kNs] = (uint8_t)((version << 1) | 1);
  memset(out + kNs + 1, 0, kShare - kNs - 1);
}

// shares.CompactShareCounter (counter.go): compact shares a run of delimited units needs
struct CompactCounter {
  uint64_t last_shares = 0, last_rem = 0, shares = 0, rem = 0;
  int64_t add(uint64_t len) {
    uint64_t d = len + uvarint_len(len);
    last_rem = rem;
    last_shares = shares;
    if (shares == 0) {
      if (d >= kFirstCompact - rem) {
        d -= kFirstCompact - rem;
        shares++;
        rem = 0;
      } else {
        rem += d;
        d = 0;
      }
    }
    if (d >= kContCompact - rem) {
      d -= kContCompact - rem;
      shares++;
      rem = 0;
    } else {
      rem += d;
      d = 0;
    }
    if (d > 0) {
      shares += d / kContCompact;
      rem = d % kContCompact;
    }
    int64_t diff = (int64_t)shares - (int64_t)last_shares;
    if (last_rem == 0 && rem > 0) diff++;
    else if (last_rem > 0 && rem == 0) diff--;
    return diff;
  }
  void revert() {
    shares = last_shares;
    rem = last_rem;
  }
  uint64_t size() const { return rem == 0 ? shares : shares + 1; }
};

// shares.CompactShareSplitter: length-delimited units into compact shares
// (ns | info | [sequence len] | reserved = offset of the first unit starting
// in the share | data), written into an internal buffer.
class CompactWriter {
 public:
  explicit CompactWriter(const Ns& ns) : ns_(ns) { start(true); }
  void write_tx(Span tx) {
    uint8_t delim[10];
    const size_t dl = put_uvarint(delim, tx.n);
    // maybe_write_reserved_bytes: the first unit that starts in this share
    if (get_be32(cur_ + reserved_at()) == 0) put_be32(cur_ + reserved_at(), (uint32_t)len_);
    add(delim, dl);
    add(tx.p, tx.n);
    if (len_ == kShare) stack();
  }
  size_t count() const { return shares_.size() / kShare + (empty_share() ? 0 : 1); }
  // Export: zero-pads the last share and writes the sequence length
  void export_to(uint8_t* out) {
    if (shares_.empty() && empty_share()) return;
    size_t padding = 0;
    if (!empty_share()) {
      padding = kShare - len_;
      memset(cur_ + len_, 0, padding);
      len_ = kShare;
      stack();
    }
    const size_t n = shares_.size() / kShare;
    const size_t seq = kFirstCompact + (n - 1) * kContCompact - padding;
    put_be32(shares_.data() + kNs + 1, (uint32_t)seq);
    memcpy(out, shares_.data(), shares_.size());
  }

 private:
  Ns ns_;
  std::vector<uint8_t> shares_;
  uint8_t cur_[kShare];
  size_t len_ = 0;
  bool first_ = true;
  size_t reserved_at() const { return kNs + 1 + (first_ ? 4 : 0); }
  bool empty_share() const { return len_ == reserved_at() + 4; }
  void start(bool first) {
    first_ = first;
    memcpy(cur_, ns_.b, kNs);
    cur_[kNs] = first ? 1 : 0;  // share version 0
    len_ = kNs + 1;
    if (first) {
      memset(cur_ + len_, 0, 4);
      len_ += 4;
    }
    memset(cur_ + len_, 0, 4);
    len_ += 4;
  }
  void stack() {
    shares_.insert(shares_.end(), cur_, cur_ + kShare);
    start(false);
  }
  void add(const uint8_t* p, size_t n) {
    while (n) {
      if (len_ == kShare) stack();
      const size_t t = std::min(n, kShare - len_);
      memcpy(cur_ + len_, p, t);
      len_ += t;
      p += t;
      n -= t;
    }
  }
};

struct Element {
  BlobRef blob;
  size_t pfb_index, blob_index;
  uint64_t num_shares, max_padding;
  uint8_t ns[kNs];
};

struct PfbRec {
  Span tx;
  std::vector<uint32_t> share_indexes;
};

// pkg/square Builder
class SquareBuilder {
 public:
  SquareBuilder(uint64_t max_square_size, uint64_t threshold) : threshold_(threshold) {
    if (max_square_size == 0) throw SquareError{"max square size must be strictly positive"};
    if (max_square_size & (max_square_size - 1)) throw SquareError{"max square size must be a power of two"};
    max_capacity_ = max_square_size * max_square_size;
  }
  bool append_tx(Span tx) {
    const int64_t diff = tx_counter_.add(tx.n);
    if (fits(diff)) {
      txs_.push_back(tx);
      current_ += diff;
      return true;
    }
    tx_counter_.revert();
    return false;
  }
  bool append_blob_tx(Span inner, const std::vector<BlobRef>& blobs) {
    // worst case: every share index is SquareSizeUpperBound^2
    const size_t iw = index_wrapper_size(inner.n, blobs.size(), 128u * 128u);
    const int64_t pfb_diff = pfb_counter_.add(iw);
    int64_t max_blob = 0;
    std::vector<Element> el;
    for (size_t i = 0; i < blobs.size(); i++) {
      Element e{};
      e.blob = blobs[i];
      e.pfb_index = pfbs_.size();
      e.blob_index = i;
      e.num_shares = sparse_shares_needed(blobs[i].data.n);
      e.max_padding = subtree_width_u(e.num_shares, threshold_) - 1;
      e.ns[0] = (uint8_t)blobs[i].ns_version;
      memcpy(e.ns + 1, blobs[i].ns_id.p, kNsId);
      max_blob += (int64_t)(e.num_shares + e.max_padding);
      el.push_back(e);
    }
    if (fits(pfb_diff + max_blob)) {
      blobs_.insert(blobs_.end(), el.begin(), el.end());
      pfbs_.push_back({inner, std::vector<uint32_t>(blobs.size(), 128u * 128u)});
      current_ += pfb_diff + max_blob;
      return true;
    }
    pfb_counter_.revert();
    return false;
  }
  bool empty() const { return tx_counter_.size() == 0 && pfb_counter_.size() == 0; }
  // square size of the export (1 for the empty square)
  uint64_t square_size() const { return empty() ? 1 : blob_min_square_size((uint64_t)current_); }

  // Export + WriteSquare into out (square_size()^2 shares)
  void export_to(uint8_t* out) {
    const uint64_t ss = square_size();
    const uint64_t total = ss * ss;
    if (empty()) {
      padding_share(out, kTailPaddingNs.b, 0);
      return;
    }
    std::stable_sort(blobs_.begin(), blobs_.end(),
                     [](const Element& a, const Element& b) { return memcmp(a.ns, b.ns, kNs) < 0; });
    CompactWriter txw(kTxNs);
    for (const Span& t : txs_) txw.write_tx(t);
    uint64_t non_reserved_start = tx_counter_.size() + pfb_counter_.size();
    uint64_t cursor = non_reserved_start, end_of_last = non_reserved_start;
    std::vector<uint64_t> start(blobs_.size());
    for (size_t i = 0; i < blobs_.size(); i++) {
      Element& e = blobs_[i];
      const uint64_t wdt = subtree_width_u(e.num_shares, threshold_);
      cursor = cursor % wdt == 0 ? cursor : (cursor / wdt + 1) * wdt;  // NextShareIndex
      if (i == 0) non_reserved_start = cursor;
      const uint64_t padding = cursor - end_of_last;
      if (padding > e.max_padding)
        throw SquareError{"blob has " + std::to_string(padding) + " padding shares, but " +
                          std::to_string(e.max_padding) + " was the max possible"};
      pfbs_[e.pfb_index].share_indexes[e.blob_index] = (uint32_t)cursor;
      start[i] = cursor;
      // the checks SparseShareSplitter makes while writing, in its order:
      // padding in the previous blob's namespace, then Blob.ValidateBasic
      if (i > 0 && padding > 0) validate_namespace(blobs_[i - 1].ns);
      if (e.blob.share_version > 255) throw SquareError{"share version can not be greater than MaxShareVersion"};
      if (e.blob.ns_version > 255)
        throw SquareError{"namespace version can not be greater than MaxNamespaceVersion"};
      if (e.blob.data.n == 0) throw SquareError{"blob data can not be empty"};
      if (e.blob.share_version != 0)
        throw SquareError{"unsupported share version: " + std::to_string(e.blob.share_version)};
      cursor += e.num_shares;
      end_of_last = cursor;
    }
    CompactWriter pfbw(kPfbNs);
    std::vector<uint8_t> iw;
    for (const PfbRec& p : pfbs_) {
      marshal_index_wrapper(p.tx, p.share_indexes, iw);
      pfbw.write_tx({iw.data(), iw.size()});
    }
    if (pfb_counter_.size() < pfbw.count())
      throw SquareError{"pfbCounter.Size() < pfbTxWriter.Count(): " + std::to_string(pfb_counter_.size()) +
                        " < " + std::to_string(pfbw.count())};
    // WriteSquare
    const uint64_t pfb_start = txw.count();
    const uint64_t padding_start = pfb_start + pfbw.count();
    if (non_reserved_start < padding_start)
      throw SquareError{"nonReservedStart " + std::to_string(non_reserved_start) +
                        " is too small to fit all PFBs and txs"};
    uint64_t blob_count = 0;
    for (size_t i = 0; i < blobs_.size(); i++) {
      blob_count += blobs_[i].num_shares;
      if (i > 0) blob_count += start[i] - (start[i - 1] + blobs_[i - 1].num_shares);
    }
    const uint64_t end_of_last_blob = non_reserved_start + blob_count;
    if (total < end_of_last_blob)
      throw SquareError{"square size " + std::to_string(total) + " is too small to fit all blobs"};
    if (blobs_.empty() && non_reserved_start != padding_start)
      throw SquareError{"square has unwritten shares"};
    txw.export_to(out);
    pfbw.export_to(out + pfb_start * kShare);
    if (!blobs_.empty()) {
      for (uint64_t s = padding_start; s < non_reserved_start; s++)
        padding_share(out + s * kShare, kReservedPaddingNs.b, 0);
      uint8_t* o = out + non_reserved_start * kShare;
      for (size_t i = 0; i < blobs_.size(); i++) {
        const Element& e = blobs_[i];
        if (i > 0) {  // namespace padding in the previous blob's namespace
          const uint64_t pad = start[i] - (start[i - 1] + blobs_[i - 1].num_shares);
          for (uint64_t p = 0; p < pad; p++, o += kShare) padding_share(o, blobs_[i - 1].ns, 0);
        }
        o = write_blob(o, e);
      }
    }
    for (uint64_t s = end_of_last_blob; s < total; s++) padding_share(out + s * kShare, kTailPaddingNs.b, 0);
  }

 private:
  uint64_t threshold_, max_capacity_ = 0;
  int64_t current_ = 0;
  CompactCounter tx_counter_, pfb_counter_;
  std::vector<Span> txs_;
  std::vector<PfbRec> pfbs_;
  std::vector<Element> blobs_;

  bool fits(int64_t n) const { return current_ + n <= (int64_t)max_capacity_; }

  // SparseShareSplitter.Write: first share ns | info | sequence len | data,
  // continuation shares ns | info | data, the last zero-padded
  static uint8_t* write_blob(uint8_t* o, const Element& e) {
    const uint8_t* p = e.blob.data.p;
    size_t n = e.blob.data.n;
    bool first = true;
    while (true) {
      memcpy(o, e.ns, kNs);
      o[kNs] = first ? 1 : 0;
      size_t at = kNs + 1;
      if (first) {
        put_be32(o + at, (uint32_t)e.blob.data.n);
        at += 4;
      }
      const size_t t = std::min(n, kShare - at);
      memcpy(o + at, p, t);
      memset(o + at + t, 0, kShare - at - t);
      o += kShare;
      p += t;
      n -= t;
      first = false;
      if (n == 0) return o;
    }
  }
};

std::vector<Span> split_txs(const uint8_t* txs, const uint64_t* lens, size_t ntx) {
  std::vector<Span> v(ntx);
  size_t off = 0;
  for (size_t i = 0; i < ntx; i++) {
    v[i] = {txs + off, (size_t)lens[i]};
    off += (size_t)lens[i];
  }
  return v;
}

int finish(dagpu_ctx* ctx, SquareBuilder& b, uint8_t* ods_out, size_t ods_cap, uint32_t* square_size) {
  const uint64_t k = b.square_size();
  if (square_size) *square_size = (uint32_t)k;
  const size_t need = (size_t)(k * k) * kShare;
  if (!ods_out || ods_cap < need)
    return set_err(ctx, DAGPU_ERR_ARG, "ods buffer too small: need " + std::to_string(need) + " bytes");
  b.export_to(ods_out);
  return DAGPU_OK;
}

}  // namespace

extern "C" {

int dagpu_square_construct(dagpu_ctx* ctx, const uint8_t* txs, const uint64_t* tx_lens, size_t ntx,
                           uint32_t max_square_size, uint32_t subtree_root_threshold, uint8_t* ods_out,
                           size_t ods_cap, uint32_t* square_size) {
  if (ntx && (!txs || !tx_lens)) return set_err(ctx, DAGPU_ERR_ARG, "txs and tx_lens are required when ntx > 0");
  if (subtree_root_threshold == 0) return set_err(ctx, DAGPU_ERR_ARG, "subtree_root_threshold must be > 0");
  try {
    SquareBuilder b(max_square_size, subtree_root_threshold);
    const std::vector<Span> v = split_txs(txs, tx_lens, ntx);
    std::vector<BlobRef> blobs;
    bool seen_blob = false;
    for (size_t i = 0; i < ntx; i++) {
      Span inner;
      if (unmarshal_blob_tx(v[i], inner, blobs)) {
        seen_blob = true;
        if (!b.append_blob_tx(inner, blobs))
          throw SquareError{"not enough space to append blob tx at index " + std::to_string(i)};
      } else {
        if (seen_blob)
          throw SquareError{"normal tx at index " + std::to_string(i) + " can not be appended after blob tx"};
        if (!b.append_tx(v[i])) throw SquareError{"not enough space to append tx at index " + std::to_string(i)};
      }
    }
    return finish(ctx, b, ods_out, ods_cap, square_size);
  } catch (const SquareError& e) {
    return set_err(ctx, DAGPU_ERR_SQUARE, e.msg);
  } catch (const std::bad_alloc&) {
    return set_err(ctx, DAGPU_ERR_SQUARE, "out of host memory");
  }
}

int dagpu_square_build(dagpu_ctx* ctx, const uint8_t* txs, const uint64_t* tx_lens, size_t ntx,
                       uint32_t max_square_size, uint32_t subtree_root_threshold, uint8_t* ods_out,
                       size_t ods_cap, uint32_t* square_size, uint8_t* kept) {
  if (ntx && (!txs || !tx_lens)) return set_err(ctx, DAGPU_ERR_ARG, "txs and tx_lens are required when ntx > 0");
  if (subtree_root_threshold == 0) return set_err(ctx, DAGPU_ERR_ARG, "subtree_root_threshold must be > 0");
  try {
    SquareBuilder b(max_square_size, subtree_root_threshold);
    const std::vector<Span> v = split_txs(txs, tx_lens, ntx);
    std::vector<BlobRef> blobs;
    for (size_t i = 0; i < ntx; i++) {
      Span inner;
      const bool ok = unmarshal_blob_tx(v[i], inner, blobs) ? b.append_blob_tx(inner, blobs) : b.append_tx(v[i]);
      if (kept) kept[i] = ok ? 1 : 0;
    }
    return finish(ctx, b, ods_out, ods_cap, square_size);
  } catch (const SquareError& e) {
    return set_err(ctx, DAGPU_ERR_SQUARE, e.msg);
  } catch (const std::bad_alloc&) {
    return set_err(ctx, DAGPU_ERR_SQUARE, "out of host memory");
  }
}

}  // extern "C"
