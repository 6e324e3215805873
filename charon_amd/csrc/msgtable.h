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

// byte equality of two messages of length l (32-byte signing roots: four word compares)
inline bool msg_eq(const uint8_t* a, const uint8_t* b, uint32_t l) {
  if (l == 32) {
    uint64_t x[4], y[4];
    memcpy(x, a, 32);
    memcpy(y, b, 32);
    return ((x[0] ^ y[0]) | (x[1] ^ y[1]) | (x[2] ^ y[2]) | (x[3] ^ y[3])) == 0;
  }
  return memcmp(a, b, l) == 0;
}

// distinct messages of the items (open addressing on item indices: no per-message allocation).
// The table starts small and doubles when half full (a slot's million partials over 100 k
// messages touch a 1 MB table, not a 2 n-slot one: fresh pages, not probes, dominated the time),
// and a run of items over one message reuses the previous item's id without a lookup.
inline void dedup_messages(const uint8_t* msgs, const uint64_t* off, const uint32_t* len, size_t n, const size_t* items,
                           MsgTable& t) {
  size_t cap = 1024;
  std::vector<uint32_t> slot(cap, 0xffffffffu);  // distinct-message id, or empty
  std::vector<uint64_t> src;                      // first item of each distinct message
  std::vector<uint64_t> hsrc;                     // its hash (rehashing without the bytes)
  t.idx.resize(n);
  for (size_t k = 0; k < n; k++) {
    const size_t i = items ? items[k] : k;
    const uint8_t* m = msgs + off[i];
    const uint32_t l = len[i];
    if (k) {  // runs of one message (a validator's partials side by side): the previous item's id
      const size_t i0 = items ? items[k - 1] : k - 1;
      if (len[i0] == l && (off[i0] == off[i] || msg_eq(msgs + off[i0], m, l))) {
        t.idx[k] = t.idx[k - 1];
        continue;
      }
    }
    const uint64_t hv = msg_hash(m, l);
    size_t h = (size_t)hv & (cap - 1);
    uint32_t id;
    for (;;) {
      id = slot[h];
      if (id == 0xffffffffu) break;
      const uint64_t j = src[id];
      if (hsrc[id] == hv && len[j] == l && msg_eq(msgs + off[j], m, l)) break;
      h = (h + 1) & (cap - 1);
    }
    if (id == 0xffffffffu) {
      id = (uint32_t)t.len.size();
      src.push_back(i);
      hsrc.push_back(hv);
      t.off.push_back(t.bytes.size());
      t.len.push_back(l);
      t.bytes.insert(t.bytes.end(), m, m + l);
      if (2 * src.size() > cap) {  // grow: re-insert every id by its hash
        cap *= 2;
        slot.assign(cap, 0xffffffffu);
        for (uint32_t q = 0; q < (uint32_t)src.size(); q++) {
          size_t g = (size_t)hsrc[q] & (cap - 1);
          while (slot[g] != 0xffffffffu) g = (g + 1) & (cap - 1);
          slot[g] = q;
        }
      } else {
        slot[h] = id;
      }
    }
    t.idx[k] = id;
  }
}

// dedup_messages for large calls (items == nullptr): T threads each dedup a contiguous range of
// the items (runs and a local table, as dedup_messages), then one pass merges the ranges' distinct
// messages into the call's table and a parallel pass renumbers the items.  A single thread is
// bound by streaming the items' bytes and offsets (~5 ns per item); the ranges stream in parallel.
inline void dedup_messages_par(const uint8_t* msgs, const uint64_t* off, const uint32_t* len, size_t n, MsgTable& t,
                               unsigned T) {
  std::vector<MsgTable> loc(T);
  std::vector<std::vector<uint64_t>> first(T);  // per range: the global item of each local message
  auto par = [&](const std::function<void(unsigned)>& f) {
    std::vector<std::thread> th;
    for (unsigned p = 1; p < T; p++) th.emplace_back(f, p);
    f(0);
    for (auto& x : th) x.join();
  };
  par([&](unsigned p) {
    const size_t b = n * p / T, e = n * (p + 1) / T;
    std::vector<size_t> items(e - b);
    for (size_t k = b; k < e; k++) items[k - b] = k;
    dedup_messages(msgs, off, len, e - b, items.data(), loc[p]);
    // the first item of each local message (ids are assigned in first-occurrence order)
    std::vector<uint64_t>& f = first[p];
    f.reserve(loc[p].len.size());
    for (size_t k = 0; k < e - b; k++)
      if (loc[p].idx[k] == f.size()) f.push_back(b + k);
  });
  // merge: the call's table over the ranges' distinct messages, in range order
  size_t total = 0;
  for (unsigned p = 0; p < T; p++) total += first[p].size();
  std::vector<uint64_t> reps;
  reps.reserve(total);
  for (unsigned p = 0; p < T; p++) reps.insert(reps.end(), first[p].begin(), first[p].end());
  std::vector<size_t> ritems(reps.begin(), reps.end());
  MsgTable g;
  dedup_messages(msgs, off, len, reps.size(), ritems.data(), g);
  std::vector<size_t> base(T + 1, 0);
  for (unsigned p = 0; p < T; p++) base[p + 1] = base[p] + first[p].size();
  t.bytes = std::move(g.bytes);
  t.off = std::move(g.off);
  t.len = std::move(g.len);
  t.idx.resize(n);
  par([&](unsigned p) {
    const size_t b = n * p / T, e = n * (p + 1) / T;
    const uint32_t* gid = g.idx.data() + base[p];  // local id -> call id
    for (size_t k = b; k < e; k++) t.idx[k] = gid[loc[p].idx[k - b]];
  });
}

}  // namespace hb
