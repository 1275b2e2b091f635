// Host data path: AST relation planes for a batch, native C++.
//
// The reference builds, per AST in pre-order (my_ast.py:198-273), the signed ancestor distance
// matrix L (L[a][c] = depth(c) - depth(a), L[c][a] = -(that), for every ancestor a of c: the pairs
// of all root-to-leaf paths) and the sibling matrix T (T[i][j] = j_idx - i_idx between children i,
// j of one parent, antisymmetric) as fp32 (N x N) torch tensors in Python loops, then collate_fn
// encodes them as idx = clamp(raw + 75, 0, 149), mask = (raw == 0) (dataset/base_data_set.py:33-36),
// and CSE repeats them to int64 (B, 8, N, N) (module/csa_trans.py:206-211).
//
// Here one call fills the four uint8 (B, N, N) planes the kernels read (head stride 0) straight from
// the parent arrays: O(N * depth) per tree for L, O(sum of squared child counts) for T, trees split
// over `nthreads` std::threads. Nodes >= max_size are dropped (my_ast.py __sub_tree truncation keeps
// a pre-order prefix, and a prefix of a pre-order is closed under taking parents).
#include <stdint.h>
#include <string.h>

#include <algorithm>
#include <thread>
#include <vector>

#include "../../include/csa_hip.h"

namespace csa {
void set_error(const char* fmt, ...);  // thread-local error text (csa_sbm.hip)
}

namespace {

constexpr int REL_OFFSET = 75, REL_MAX = 149;

inline uint8_t rel_idx(int raw) {
  const int v = raw + REL_OFFSET;
  return (uint8_t)(v < 0 ? 0 : v > REL_MAX ? REL_MAX : v);
}

// returns false on a malformed tree (parent id not smaller than the node id)
bool one_tree(const int32_t* parent, int n, int N, uint8_t* L, uint8_t* T, uint8_t* Lm, uint8_t* Tm,
              std::vector<int>& depth, std::vector<int>& rawL, std::vector<int>& rawT, std::vector<int>& kid_start,
              std::vector<int>& kids) {
  n = std::min(n, N);
  rawL.assign((size_t)N * N, 0);
  rawT.assign((size_t)N * N, 0);
  depth.assign(n > 0 ? n : 1, 0);
  for (int v = 1; v < n; ++v) {
    const int p = parent[v];
    if (p < 0 || p >= v) return false;
    depth[v] = depth[p] + 1;
  }
  if (n > 0 && parent[0] >= 0) return false;
  for (int c = 1; c < n; ++c)
    for (int a = parent[c]; a >= 0; a = parent[a]) {
      const int d = depth[c] - depth[a];
      rawL[(size_t)a * N + c] = d;
      rawL[(size_t)c * N + a] = -d;
    }
  // children of each node in increasing (pre-order) id: counting sort by parent
  kid_start.assign(n + 1, 0);
  for (int v = 1; v < n; ++v) ++kid_start[parent[v] + 1];
  for (int p = 0; p < n; ++p) kid_start[p + 1] += kid_start[p];
  kids.assign(n > 1 ? n - 1 : 1, 0);
  {
    std::vector<int> fill(kid_start.begin(), kid_start.end() - 1);
    for (int v = 1; v < n; ++v) kids[fill[parent[v]]++] = v;
  }
  for (int p = 0; p < n; ++p) {
    const int s = kid_start[p], e = kid_start[p + 1];
    for (int i = s; i < e; ++i)
      for (int j = i + 1; j < e; ++j) {
        rawT[(size_t)kids[i] * N + kids[j]] = j - i;
        rawT[(size_t)kids[j] * N + kids[i]] = -(j - i);
      }
  }
  for (size_t e = 0; e < (size_t)N * N; ++e) {
    L[e] = rel_idx(rawL[e]);
    T[e] = rel_idx(rawT[e]);
    Lm[e] = rawL[e] == 0;
    Tm[e] = rawT[e] == 0;
  }
  return true;
}

}  // namespace

extern "C" csa_status csa_ast_relations(const int32_t* parent, const int32_t* n_nodes, int64_t B, int64_t max_size,
                                        uint8_t* L, uint8_t* T, uint8_t* L_mask, uint8_t* T_mask, int nthreads) {
  if (B < 0 || max_size < 1 || max_size > 4096) {
    csa::set_error("csa_ast_relations: bad B / max_size");
    return CSA_INVALID_ARG;
  }
  if (B == 0) return CSA_OK;
  if (!parent || !n_nodes || !L || !T || !L_mask || !T_mask) {
    csa::set_error("csa_ast_relations: null pointer");
    return CSA_INVALID_ARG;
  }
  const int N = (int)max_size;
  const size_t plane = (size_t)N * N;
  const int nt = (int)std::max<int64_t>(1, std::min<int64_t>(nthreads < 1 ? 1 : nthreads, B));
  std::vector<char> ok((size_t)B, 1);
  auto work = [&](int t) {
    std::vector<int> depth, rawL, rawT, ks, kids;
    for (int64_t b = t; b < B; b += nt) {
      const int n = n_nodes[b] < 0 ? 0 : n_nodes[b];
      ok[b] = one_tree(parent + b * max_size, n, N, L + b * plane, T + b * plane, L_mask + b * plane,
                       T_mask + b * plane, depth, rawL, rawT, ks, kids);
    }
  };
  if (nt == 1) {
    work(0);
  } else {
    std::vector<std::thread> th;
    for (int t = 0; t < nt; ++t) th.emplace_back(work, t);
    for (auto& x : th) x.join();
  }
  for (int64_t b = 0; b < B; ++b)
    if (!ok[b]) {
      csa::set_error("csa_ast_relations: tree %lld: parent ids must precede their children (pre-order)", (long long)b);
      return CSA_INVALID_ARG;
    }
  return CSA_OK;
}

// collect_fn's relation encoding (dataset/base_data_set.py:33-36) of already-built raw fp32 L / T
// matrices (the preprocessed split_matrices.npz format): idx = clamp(raw + 75, 0, 149) as uint8 and
// mask = (raw == 0), n elements, split over nthreads std::threads. Raw values are integral distances;
// the float is converted the way torch.clamp(x + 75, 0, 149) then .to(int64) rounds (toward zero).
extern "C" csa_status csa_collate_relations(const float* L_raw, const float* T_raw, int64_t n, uint8_t* L, uint8_t* T,
                                            uint8_t* L_mask, uint8_t* T_mask, int nthreads) {
  if (n < 0 || !L_raw || !T_raw || !L || !T || !L_mask || !T_mask) {
    csa::set_error("csa_collate_relations: null pointer or negative size");
    return CSA_INVALID_ARG;
  }
  const int nt = nthreads < 1 ? 1 : nthreads;
  auto enc = [](float raw) -> uint8_t {
    const float v = raw + (float)REL_OFFSET;
    const float c = v < 0.f ? 0.f : v > (float)REL_MAX ? (float)REL_MAX : v;
    return (uint8_t)(int)c;
  };
  auto work = [&](int t) {
    const int64_t lo = n * t / nt, hi = n * (t + 1) / nt;
    for (int64_t e = lo; e < hi; ++e) {
      L[e] = enc(L_raw[e]);
      T[e] = enc(T_raw[e]);
      L_mask[e] = L_raw[e] == 0.f;
      T_mask[e] = T_raw[e] == 0.f;
    }
  };
  if (nt == 1 || n < (1 << 16)) {
    for (int t = 0; t < nt; ++t) work(t);
  } else {
    std::vector<std::thread> th;
    for (int t = 0; t < nt; ++t) th.emplace_back(work, t);
    for (auto& x : th) x.join();
  }
  return CSA_OK;
}

// Build provenance: sha256 of every source and header the library was compiled from, passed in by
// csa_amd/build.py (-DCSA_SOURCE_HASH). smoke() and the tests compare it with the tree they run in.
#ifndef CSA_SOURCE_HASH
#define CSA_SOURCE_HASH "unknown"
#endif
extern "C" const char* csa_source_hash(void) { return CSA_SOURCE_HASH; }
