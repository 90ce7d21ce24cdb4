// g2n_keyset.hip — a device set of byte keys with dense ids in insertion order, grown call by
// call (g2n_keyset_*): the chunked build's file-wide dictionary of names (shard.py
// _chunked_general).  A chunk's distinct local names are looked up in the set; the new ones take
// the next ids in the chunk's order — builders.py:194-198's first-touch minting across chunks,
// since earlier chunks come first — and are appended.  Each call costs the chunk's keys, not the
// set's (the earlier form re-deduplicated the whole set with every chunk).
//
// Open addressing over 16-byte entries (hdr = hash tag << 32 | id, ~0 = empty; loc = key length
// << 40 | the key's offset in the set's blob), load <= 1/2, linear probing; a key is found by tag,
// length and its bytes.  Growing re-inserts every key from the set's own blob.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace g2n {

struct KsEntry {
  unsigned long long hdr;
  unsigned long long loc;
};
constexpr unsigned long long kKsEmpty = ~0ull;
constexpr unsigned long long kKsOffMask = (1ull << 40) - 1;
constexpr uint64_t kKsMaxKeyLen = (1ull << 24) - 1;  // loc's length field (a longer key: G2N_E_UNSUPPORTED)

__device__ inline uint64_t ks_hash(const uint8_t* __restrict__ p, uint64_t n) {  // FNV-1a, 64-bit
  uint64_t h = 0xcbf29ce484222325ull;
  for (uint64_t j = 0; j < n; j++) h = (h ^ p[j]) * 0x100000001b3ull;
  return h ^ (h >> 29);
}

// key i of (blob, offs): its id in the set, or ~0u (new: fresh[i] = 1)
__global__ void __launch_bounds__(256) k_ks_lookup(const uint8_t* __restrict__ blob, const int64_t* __restrict__ offs,
                                                   uint64_t n, const KsEntry* __restrict__ table, uint64_t mask,
                                                   const uint8_t* __restrict__ sblob, uint32_t* __restrict__ ids,
                                                   uint32_t* __restrict__ fresh) {
  const uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= n) return;
  const uint8_t* k = blob + offs[i];
  const uint64_t len = (uint64_t)(offs[i + 1] - offs[i]);
  const uint64_t h = ks_hash(k, len);
  const uint32_t tag = (uint32_t)(h >> 32);
  uint32_t id = ~0u;
  for (uint64_t idx = h & mask;; idx = (idx + 1) & mask) {
    const KsEntry e = table[idx];
    if (e.hdr == kKsEmpty) break;
    if ((uint32_t)(e.hdr >> 32) == tag && (e.loc >> 40) == len) {
      const uint8_t* s = sblob + (e.loc & kKsOffMask);
      uint64_t j = 0;
      while (j < len && s[j] == k[j]) j++;
      if (j == len) {
        id = (uint32_t)e.hdr;
        break;
      }
    }
  }
  ids[i] = id;
  fresh[i] = id == ~0u ? 1u : 0u;
}

// the new keys (fresh): id = base + their rank among the new ones (pos, exclusive scan of fresh);
// bytes appended to the set's blob at sblob_len + bpos[i] (bpos: exclusive scan of their lengths),
// their end offsets to soffs; then claimed in the table (distinct keys: no two race for one key).
// reinsert (growth): every key of the set itself, ids 0..n-1, bytes already in place.
__global__ void __launch_bounds__(256) k_ks_insert(const uint8_t* __restrict__ blob, const int64_t* __restrict__ offs,
                                                   uint64_t n, const uint32_t* __restrict__ fresh,
                                                   const uint32_t* __restrict__ pos, const int64_t* __restrict__ bpos,
                                                   uint64_t base, uint64_t sblob_len, KsEntry* __restrict__ table,
                                                   uint64_t mask, uint8_t* __restrict__ sblob, int64_t* __restrict__ soffs,
                                                   uint32_t* __restrict__ ids, int reinsert) {
  const uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= n) return;
  if (!reinsert && !fresh[i]) return;
  const uint8_t* k = blob + offs[i];
  const uint64_t len = (uint64_t)(offs[i + 1] - offs[i]);
  uint64_t at;
  uint32_t id;
  if (reinsert) {
    at = (uint64_t)offs[i];
    id = (uint32_t)i;
  } else {
    at = sblob_len + (uint64_t)bpos[i];
    id = (uint32_t)(base + pos[i]);
    for (uint64_t j = 0; j < len; j++) sblob[at + j] = k[j];
    soffs[id + 1] = (int64_t)(at + len);
    ids[i] = id;
  }
  const uint64_t h = ks_hash(k, len);
  const unsigned long long hdr = ((unsigned long long)(uint32_t)(h >> 32) << 32) | id;
  for (uint64_t idx = h & mask;; idx = (idx + 1) & mask) {
    if (atomicCAS(&table[idx].hdr, kKsEmpty, hdr) == kKsEmpty) {
      table[idx].loc = (len << 40) | at;
      break;
    }
  }
}

__global__ void __launch_bounds__(256) k_ks_new_lens(const int64_t* __restrict__ offs, const uint32_t* __restrict__ fresh,
                                                     uint64_t n, int64_t* __restrict__ lens) {
  const uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= n) return;
  lens[i] = fresh[i] ? offs[i + 1] - offs[i] : 0;
}

// the longest of n key lengths, into *out (atomicMax per block: only run when the new keys' bytes
// could hold one longer than kKsMaxKeyLen)
__global__ void __launch_bounds__(256) k_ks_max_len(const int64_t* __restrict__ lens, uint64_t n,
                                                    unsigned long long* out) {
  unsigned long long m = 0;
  for (uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (uint64_t)gridDim.x * 256)
    m = max(m, (unsigned long long)lens[i]);
  for (int o = 32; o > 0; o >>= 1) m = max(m, (unsigned long long)__shfl_xor(m, o, 64));
  if ((threadIdx.x & 63) == 0 && m) atomicMax(out, m);
}

}  // namespace g2n
