// Launchers of the evaluation kernels of kyv_kernels.h (kyv_launch.inc): kyvprod:: -- the product build
// (kyv_prod.hip, namespace kyv) -- and kyvacct:: -- the byte-accounting build (kyv_acct.hip: the same source compiled
// with KYV_ACCT in a renamed namespace). Plain types only: the argument structs are the product's (kyv::View, DevOut,
// WorkLists, ChunkMap), passed by address and copied into their layout-identical twins.
#pragma once
#include <hip/hip_runtime.h>
#include <cstdint>

#define KYV_LAUNCH_DECLS \
  void match(unsigned grid, hipStream_t s, const void* view, const void* devout, const void* wl, const uint32_t* mrules,\
             uint32_t nm);\
  void match_j(unsigned grid, hipStream_t s, const void* view, const void* devout, const void* wl, const uint32_t* mrules,\
               uint32_t nm);\
  void match_rec(int wpe, bool mw1, unsigned grid, hipStream_t s, const void* view, const void* devout, const void* wl,\
                 const void* recs, uint32_t nm, const void* index, const void* shapes, const void* tails,\
                 const void* facts);\
  void facts(bool mw1, unsigned grid, hipStream_t s, const void* view, const void* cfg, void* out);\
  void match_walk_generic(int wpe, unsigned grid, hipStream_t s, const void* view, const void* devout, const void* wl,\
                          const uint32_t* mrules, uint32_t nm);\
  void match_pre(unsigned grid, hipStream_t s, const void* view, const void* devout, const void* wl, const uint32_t* mrules,\
                 uint32_t nm);\
  void match_pre_j(unsigned grid, hipStream_t s, const void* view, const void* devout, const void* wl, const uint32_t* mrules,\
                   uint32_t nm);\
  void pss(bool exact, bool pre, int wpe, unsigned grid, hipStream_t s, const void* view, const void* devout, uint32_t k,\
           uint32_t w0);\
  void match_deny(unsigned grid, hipStream_t s, const void* view, const void* devout, const uint32_t* mrules, uint32_t nm);\
  void pss_map(unsigned grid, hipStream_t s, const void* view, const void* devout, uint32_t k, uint32_t w0);\
  void walk(unsigned grid, size_t lds, hipStream_t s, const void* view, const void* devout, const void* wl, const void* cm,\
            int depth);

namespace kyvprod {
KYV_LAUNCH_DECLS
}  // namespace kyvprod
namespace kyvacct {
KYV_LAUNCH_DECLS
// device addresses of this build's counters, one set per translation unit (kyv_acct.hip, kyv_acct_j.hip: each has its
// own code object): unsigned long long[3][KYV_ACCT_SLOTS] (reads, writes, staged records)
unsigned long long* counters();
unsigned long long* counters_j();
}  // namespace kyvacct
