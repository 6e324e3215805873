// roots.hip: the 32-byte signing roots of a slot's attestations, on device.
//
// charon builds every message it verifies as GetDataRoot(domain, object root)
// (eth2util/signing/signing.go:63-77: SSZ SigningData{object_root, domain}); for attestations the
// object root is phase0.AttestationData.HashTreeRoot (core/signeddata.go Attestation.MessageRoot,
// consensus-specs AttestationData{slot, index, beacon_block_root, source, target}).  Here one lane
// takes one AttestationData in its 128-byte SSZ encoding and writes its signing root, so the
// messages of a slot go from the wire format to hash-to-G2 without a host round trip.
//
// Merkleisation of the 5-field container (8 leaves, 3 zero):
//   c0 = slot, c1 = index, c2 = beacon_block_root, c3 = H(src.epoch, src.root), c4 = H(tgt...)
//   root = H(H(H(c0, c1), H(c2, c3)), H(H(c4, 0), Z1))      Z1 = H(0, 0)
//   signing root = H(root, domain)
// H(l, r) = SHA-256 of the 64 bytes l || r: two compressions (data block + the constant padding
// block).  8 H per attestation, i.e. 16 SHA-256 compressions: integer VALU work, negligible next
// to the pairing path (k_attestation_roots in DESIGN.md §4).
#include "layout.h"
#include "sha256.h"

namespace hb {

// a 32-byte chunk as 8 big-endian words (the SHA-256 message word order)
struct Chunk {
  uint32_t w[8];
};

__device__ __forceinline__ Chunk chunk_load(const uint8_t* p) {
  Chunk c;
  HB_UNROLL for (int i = 0; i < 8; i++)
    c.w[i] = ((uint32_t)p[4 * i] << 24) | ((uint32_t)p[4 * i + 1] << 16) | ((uint32_t)p[4 * i + 2] << 8) |
             (uint32_t)p[4 * i + 3];
  return c;
}

// uint64 little-endian in the first 8 bytes of a chunk, zero padded
__device__ __forceinline__ Chunk chunk_u64(const uint8_t* p) {
  Chunk c;
  HB_UNROLL for (int i = 0; i < 8; i++) c.w[i] = 0;
  c.w[0] = ((uint32_t)p[0] << 24) | ((uint32_t)p[1] << 16) | ((uint32_t)p[2] << 8) | (uint32_t)p[3];
  c.w[1] = ((uint32_t)p[4] << 24) | ((uint32_t)p[5] << 16) | ((uint32_t)p[6] << 8) | (uint32_t)p[7];
  return c;
}

__device__ __forceinline__ Chunk chunk_zero() {
  Chunk c;
  HB_UNROLL for (int i = 0; i < 8; i++) c.w[i] = 0;
  return c;
}

// H(l || r): SHA-256 of one 64-byte message
__device__ __forceinline__ Chunk h2(const Chunk& l, const Chunk& r) {
  uint32_t blk[16];
  HB_UNROLL for (int i = 0; i < 8; i++) {
    blk[i] = l.w[i];
    blk[8 + i] = r.w[i];
  }
  Sha256State st = sha256_init();
  sha256_compress(st, blk);
  HB_UNROLL for (int i = 0; i < 16; i++) blk[i] = 0;
  blk[0] = 0x80000000u;
  blk[15] = 512;  // message length in bits
  sha256_compress(st, blk);
  Chunk o;
  HB_UNROLL for (int i = 0; i < 8; i++) o.w[i] = st.h[i];
  return o;
}

__device__ __forceinline__ void chunk_store(uint8_t* p, const Chunk& c) {
  HB_UNROLL for (int i = 0; i < 8; i++) {
    p[4 * i] = (uint8_t)(c.w[i] >> 24);
    p[4 * i + 1] = (uint8_t)(c.w[i] >> 16);
    p[4 * i + 2] = (uint8_t)(c.w[i] >> 8);
    p[4 * i + 3] = (uint8_t)c.w[i];
  }
}

// One lane per attestation: data[i] (128 B SSZ) -> roots[i] = GetDataRoot(domains[dom_idx[i]], HTR)
__global__ __launch_bounds__(64) void k_attestation_roots(const uint8_t* __restrict__ data, uint32_t n,
                                                         const uint8_t* __restrict__ domains, uint32_t n_domains,
                                                         const uint32_t* __restrict__ dom_idx,
                                                         uint8_t* __restrict__ roots) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const uint8_t* a = data + 128ull * i;
  const Chunk z = chunk_zero();
  const Chunk src = h2(chunk_u64(a + 48), chunk_load(a + 56));
  const Chunk tgt = h2(chunk_u64(a + 88), chunk_load(a + 96));
  const Chunk n01 = h2(chunk_u64(a + 0), chunk_u64(a + 8));
  const Chunk n23 = h2(chunk_load(a + 16), src);
  const Chunk n45 = h2(tgt, z);
  const Chunk n67 = h2(z, z);
  const Chunk root = h2(h2(n01, n23), h2(n45, n67));
  const uint32_t d = dom_idx ? dom_idx[i] : 0u;
  // an out-of-range domain index (validated on the host for host-buffer calls) yields the all-zero
  // root, never a root under another domain: no signature over a real signing root verifies on it
  chunk_store(roots + 32ull * i, d < n_domains ? h2(root, chunk_load(domains + 32ull * d)) : chunk_zero());
}

// One lane per object root: roots[i] = SigningData{object_roots[i], domains[dom_idx[i]]}.HTR
__global__ __launch_bounds__(64) void k_signing_roots(const uint8_t* __restrict__ obj, uint32_t n,
                                                     const uint8_t* __restrict__ domains, uint32_t n_domains,
                                                     const uint32_t* __restrict__ dom_idx,
                                                     uint8_t* __restrict__ roots) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const uint32_t d = dom_idx ? dom_idx[i] : 0u;
  chunk_store(roots + 32ull * i,
              d < n_domains ? h2(chunk_load(obj + 32ull * i), chunk_load(domains + 32ull * d)) : chunk_zero());
}

// ---- the other duty types (core/signeddata.go MessageRoot): one lane per object, its SSZ bytes
// at data[off[i] .. off[i] + len[i]); the object root, then the signing root under its domain.
// A malformed object (length, offsets, bitlist) gets status HBLS_BAD_INPUT and the all-zero root.
//   kind 1 phase0.AggregateAndProof (SignedAggregateAndProof, :979): aggregator_index, offset of
//          the aggregate, selection_proof; aggregate = Attestation{offset of aggregation_bits
//          (Bitlist[2048]), AttestationData, signature}, then the bits with their delimiter
//   kind 2 altair.ContributionAndProof (SignedSyncContributionAndProof, :1227): 264 bytes
//   kind 3 altair.SyncAggregatorSelectionData{slot, subcommittee_index} (SyncContributionAndProof /
//          SyncCommitteeSelection, :1135 / :915): 16 bytes
//   kind 4 a uint64 slot (BeaconCommitteeSelection, :852, eth2util.SlotHashRoot): 8 bytes
//   kind 5 the beacon block root (SignedSyncMessage, :1056): 32 bytes, the object root itself
//   kind 6 v1.ValidatorRegistration{fee_recipient, gas_limit, timestamp, pubkey}
//          (VersionedSignedValidatorRegistration, :661): 84 bytes
//   kind 7 phase0.VoluntaryExit{epoch, validator_index} (SignedVoluntaryExit, :580): 16 bytes
//   kind 8 the uint64 epoch of eth2util.SignedEpoch (SignedRandao, :791): 8 bytes
//   kind 9 phase0.BeaconBlockHeader{slot, proposer_index, parent_root, state_root, body_root}
//          (VersionedSignedProposal, :301): 112 bytes -- a block's hash-tree-root is its header's,
//          so the caller passes the block body's root (every version's block shares this shape)
__device__ __forceinline__ uint32_t rd_u32le(const uint8_t* p) {
  return (uint32_t)p[0] | ((uint32_t)p[1] << 8) | ((uint32_t)p[2] << 16) | ((uint32_t)p[3] << 24);
}
// AttestationData (128 B): the 5-field container of k_attestation_roots
__device__ __forceinline__ Chunk att_data_root(const uint8_t* a) {
  const Chunk z = chunk_zero();
  const Chunk src = h2(chunk_u64(a + 48), chunk_load(a + 56));
  const Chunk tgt = h2(chunk_u64(a + 88), chunk_load(a + 96));
  return h2(h2(h2(chunk_u64(a + 0), chunk_u64(a + 8)), h2(chunk_load(a + 16), src)), h2(h2(tgt, z), h2(z, z)));
}
// a 96-byte signature: three chunks merkleized to four
__device__ __forceinline__ Chunk sig_root(const uint8_t* p) {
  return h2(h2(chunk_load(p), chunk_load(p + 32)), h2(chunk_load(p + 64), chunk_zero()));
}
// chunk k of a byte string of length n (zero beyond n), with the byte at `clear_at` cleared of bit
// `clear_bit` (the bitlist delimiter)
__device__ __forceinline__ Chunk chunk_bytes(const uint8_t* p, uint32_t n, uint32_t k, uint32_t clear_at,
                                             uint32_t clear_mask) {
  Chunk c;
  HB_UNROLL for (int w = 0; w < 8; w++) {
    uint32_t v = 0;
    HB_UNROLL for (int j = 0; j < 4; j++) {
      const uint32_t at = 32 * k + 4 * w + j;
      uint32_t byte = at < n ? p[at] : 0u;
      if (at == clear_at) byte &= ~clear_mask;
      v = (v << 8) | byte;
    }
    c.w[w] = v;
  }
  return c;
}
// Bitlist[2048] from its encoding (b, nb bytes, the last holding the delimiter): merkleize the
// eight chunks of the limit, mix in the bit length.  false if malformed.
__device__ __forceinline__ bool bitlist2048_root(const uint8_t* b, uint32_t nb, Chunk& out) {
  if (nb < 1 || nb > 257) return false;
  const uint32_t last = b[nb - 1];
  if (last == 0) return false;
  const uint32_t top = 31u - __builtin_clz(last);  // the delimiter's bit
  const uint32_t nbits = 8 * (nb - 1) + top;
  if (nbits > 2048) return false;
  Chunk c[8];
  HB_UNROLL for (uint32_t k = 0; k < 8; k++) c[k] = chunk_bytes(b, nb, k, nb - 1, 1u << top);
  const Chunk r = h2(h2(h2(c[0], c[1]), h2(c[2], c[3])), h2(h2(c[4], c[5]), h2(c[6], c[7])));
  Chunk len = chunk_zero();  // uint256 little-endian length
  len.w[0] = ((nbits & 0xffu) << 24) | ((nbits >> 8 & 0xffu) << 16);
  out = h2(r, len);
  return true;
}
__global__ __launch_bounds__(64) void k_duty_roots(int kind, const uint8_t* __restrict__ data,
                                                  const uint64_t* __restrict__ off, const uint32_t* __restrict__ len,
                                                  uint32_t n, const uint8_t* __restrict__ domains, uint32_t n_domains,
                                                  const uint32_t* __restrict__ dom_idx, uint8_t* __restrict__ roots,
                                                  uint8_t* __restrict__ status) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const uint8_t* p = data + off[i];
  const uint32_t L = len[i];
  const Chunk z = chunk_zero();
  Chunk root = z;
  bool ok = false;
  if (kind == 1 && L >= 108 + 228 + 1 && rd_u32le(p + 8) == 108) {
    const uint8_t* att = p + 108;
    Chunk bits;
    if (rd_u32le(att) == 228 && bitlist2048_root(att + 228, L - 108 - 228, bits)) {
      const Chunk att_root = h2(h2(bits, att_data_root(att + 4)), h2(sig_root(att + 132), z));
      root = h2(h2(chunk_u64(p), att_root), h2(sig_root(p + 12), z));
      ok = true;
    }
  } else if (kind == 2 && L == 264) {
    const uint8_t* c = p + 8;
    const Chunk contrib = h2(h2(h2(chunk_u64(c), chunk_load(c + 8)), h2(chunk_u64(c + 40), chunk_bytes(c + 48, 16, 0, ~0u, 0))),
                             h2(h2(sig_root(c + 64), z), h2(z, z)));
    root = h2(h2(chunk_u64(p), contrib), h2(sig_root(p + 168), z));
    ok = true;
  } else if (kind == 3 && L == 16) {
    root = h2(chunk_u64(p), chunk_u64(p + 8));
    ok = true;
  } else if (kind == 4 && L == 8) {
    root = chunk_u64(p);
    ok = true;
  } else if (kind == 5 && L == 32) {
    root = chunk_load(p);
    ok = true;
  } else if (kind == 6 && L == 84) {
    // Bytes20 fee recipient (one chunk, zero padded), two uint64, the 48-byte key as two chunks
    const Chunk pk = h2(chunk_load(p + 36), chunk_bytes(p + 68, 16, 0, ~0u, 0));
    root = h2(h2(chunk_bytes(p, 20, 0, ~0u, 0), chunk_u64(p + 20)), h2(chunk_u64(p + 28), pk));
    ok = true;
  } else if (kind == 7 && L == 16) {
    root = h2(chunk_u64(p), chunk_u64(p + 8));
    ok = true;
  } else if (kind == 8 && L == 8) {
    root = chunk_u64(p);
    ok = true;
  } else if (kind == 9 && L == 112) {
    root = h2(h2(h2(chunk_u64(p), chunk_u64(p + 8)), h2(chunk_load(p + 16), chunk_load(p + 48))),
              h2(h2(chunk_load(p + 80), z), h2(z, z)));
    ok = true;
  }
  const uint32_t d = dom_idx ? dom_idx[i] : 0u;
  ok = ok && d < n_domains;
  chunk_store(roots + 32ull * i, ok ? h2(root, chunk_load(domains + 32ull * d)) : z);
  status[i] = ok ? 0 : 6;  // HBLS_BAD_INPUT
}

void launch_duty_roots(int kind, const uint8_t* data, const uint64_t* off, const uint32_t* len, uint32_t n,
                       const uint8_t* domains, uint32_t n_domains, const uint32_t* dom_idx, uint8_t* roots,
                       uint8_t* status, hipStream_t s) {
  if (n)
    hipLaunchKernelGGL(k_duty_roots, dim3((n + 63) / 64), dim3(64), 0, s, kind, data, off, len, n, domains, n_domains,
                       dom_idx, roots, status);
}

void launch_attestation_roots(const uint8_t* data, uint32_t n, const uint8_t* domains, uint32_t n_domains,
                              const uint32_t* dom_idx, uint8_t* roots, hipStream_t s) {
  if (n)
    hipLaunchKernelGGL(k_attestation_roots, dim3((n + 63) / 64), dim3(64), 0, s, data, n, domains, n_domains,
                       dom_idx, roots);
}
void launch_signing_roots(const uint8_t* obj, uint32_t n, const uint8_t* domains, uint32_t n_domains,
                          const uint32_t* dom_idx, uint8_t* roots, hipStream_t s) {
  if (n)
    hipLaunchKernelGGL(k_signing_roots, dim3((n + 63) / 64), dim3(64), 0, s, obj, n, domains, n_domains, dom_idx,
                       roots);
}

}  // namespace hb
