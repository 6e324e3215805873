// Host-side message tables of the host-buffer Verify calls (hipbls.hip verify_host): the distinct
// messages of a batch and each item's message id.  Host code only (no HIP), also compiled into
// the CPU test harness (tests/native/hostcheck.cpp hc_dedup: the parallel dedup partitions the
// items exactly as the sequential one).
#pragma once
#include <stdint.h>
#include <string.h>

#include <functional>
#include <thread>
#include <vector>

namespace hb {

struct MsgTable {
  std::vector<uint8_t> bytes;
  std::vector<uint64_t> off;
  std::vector<uint32_t> len;
  std::vector<uint32_t> idx;  // per item
};

// 64-bit words of the message folded by multiply-xorshift steps (messages are usually 32-byte
// signing roots, already uniform: four steps instead of FNV's 32 byte-wise multiplies)
inline uint64_t msg_hash(const uint8_t* p, uint32_t n) {
  uint64_t h = 0xcbf29ce484222325ull ^ n;
  uint32_t k = 0;
  for (; k + 8 <= n; k += 8) {
    uint64_t w;
    memcpy(&w, p + k, 8);
    h = (h ^ w) * 0x9e3779b97f4a7c15ull;
    h ^= h >> 31;
  }
  for (; k < n; k++) h = (h ^ p[k]) * 0x100000001b3ull;
  h ^= h >> 29;
  h *= 0xbf58476d1ce4e5b9ull;
  return h ^ (h >> 32);
}

// distinct messages of the items (open addressing on item indices: no per-message allocation;
// a slot's million host-buffer partials dedup in a few milliseconds)
inline void dedup_messages(const uint8_t* msgs, const uint64_t* off, const uint32_t* len, size_t n, const size_t* items,
                    MsgTable& t) {
  size_t cap = 16;
  while (cap < 2 * n + 2) cap <<= 1;
  std::vector<uint32_t> slot(cap, 0xffffffffu);  // distinct-message id, or empty
  std::vector<uint64_t> src;                      // first item of each distinct message
  t.idx.resize(n);
  for (size_t k = 0; k < n; k++) {
    const size_t i = items ? items[k] : k;
    const uint8_t* m = msgs + off[i];
    const uint32_t l = len[i];
    size_t h = (size_t)msg_hash(m, l) & (cap - 1);
    uint32_t id;
    for (;;) {
      id = slot[h];
      if (id == 0xffffffffu) break;
      const uint64_t j = src[id];
      if (len[j] == l && memcmp(msgs + off[j], m, l) == 0) break;
      h = (h + 1) & (cap - 1);
    }
    if (id == 0xffffffffu) {
      id = (uint32_t)t.len.size();
      slot[h] = id;
      src.push_back(i);
      t.off.push_back(t.bytes.size());
      t.len.push_back(l);
      t.bytes.insert(t.bytes.end(), m, m + l);
    }
    t.idx[k] = id;
  }
}

// dedup_messages for large calls (items == nullptr): the messages' hashes in parallel, then one
// thread per partition of the hash space (its top bits) runs the open-addressing dedup of its own
// items, ids offset by the partitions before it.  The ids come out in partition order instead of
// first-occurrence order -- any consistent numbering serves (items are sorted by id next).
inline void dedup_messages_par(const uint8_t* msgs, const uint64_t* off, const uint32_t* len, size_t n, MsgTable& t,
                        unsigned T) {
  std::vector<uint64_t> hs(n);
  std::vector<uint32_t> loc(n);
  auto par = [&](const std::function<void(unsigned)>& f) {
    std::vector<std::thread> th;
    for (unsigned p = 1; p < T; p++) th.emplace_back(f, p);
    f(0);
    for (auto& x : th) x.join();
  };
  par([&](unsigned p) {
    for (size_t k = n * p / T; k < n * (p + 1) / T; k++) hs[k] = msg_hash(msgs + off[k], len[k]);
  });
  const unsigned bits = 31 - __builtin_clz(T);  // T a power of two: partition = top `bits` bits
  std::vector<std::vector<uint64_t>> first(T);  // per partition: the first item of each local message
  par([&](unsigned p) {
    size_t cnt = 0;
    for (size_t k = 0; k < n; k++) cnt += (bits ? (hs[k] >> (64 - bits)) : 0) == p;
    size_t cap = 16;
    while (cap < 2 * cnt + 2) cap <<= 1;
    std::vector<uint32_t> slot(cap, 0xffffffffu);
    std::vector<uint64_t>& src = first[p];
    for (size_t k = 0; k < n; k++) {
      if ((bits ? (hs[k] >> (64 - bits)) : 0) != p) continue;
      const uint8_t* m = msgs + off[k];
      const uint32_t l = len[k];
      size_t h = (size_t)hs[k] & (cap - 1);
      uint32_t id;
      for (;;) {
        id = slot[h];
        if (id == 0xffffffffu) break;
        const uint64_t j = src[id];
        if (len[j] == l && memcmp(msgs + off[j], m, l) == 0) break;
        h = (h + 1) & (cap - 1);
      }
      if (id == 0xffffffffu) {
        id = (uint32_t)src.size();
        slot[h] = id;
        src.push_back(k);
      }
      loc[k] = id;
    }
  });
  std::vector<size_t> base(T + 1, 0), bbase(T + 1, 0);
  for (unsigned p = 0; p < T; p++) {
    base[p + 1] = base[p] + first[p].size();
    size_t bytes = 0;
    for (uint64_t j : first[p]) bytes += len[j];
    bbase[p + 1] = bbase[p] + bytes;
  }
  t.idx.resize(n);
  t.off.resize(base[T]);
  t.len.resize(base[T]);
  t.bytes.resize(bbase[T]);
  par([&](unsigned p) {
    size_t b = bbase[p];
    for (size_t q = 0; q < first[p].size(); q++) {
      const uint64_t j = first[p][q];
      t.off[base[p] + q] = b;
      t.len[base[p] + q] = len[j];
      memcpy(t.bytes.data() + b, msgs + off[j], len[j]);
      b += len[j];
    }
    for (size_t k = n * p / T; k < n * (p + 1) / T; k++)
      t.idx[k] = (uint32_t)(base[bits ? (hs[k] >> (64 - bits)) : 0] + loc[k]);
  });
}

}  // namespace hb
