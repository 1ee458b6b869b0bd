// midaspom_amd/csrc/spom_jit.h -- problem-specialised forward kernel (hipRTC).
#ifndef SPOM_JIT_H
#define SPOM_JIT_H
#include <cstddef>
#include <cstdint>
#include <string>
#include <vector>

struct MdpJitPlan {
    std::vector<uint32_t> np;     // possible states per year
    std::vector<uint32_t> udesc;  // per forward use: Q offset | nX << 22 | nA << 27
    size_t ldQ = 0;               // Q block in LDS (doubles, even)
    size_t ncoef = 0;             // Q entries assembled from the colonisation factors
    size_t ldP = 0;               // per-c colonisation-factor row Pc[c][item] (doubles, even)
    size_t nqi = 0;               // length of the Q-assembly item list (qitem)
    int epl = 0;                  // grid points per lane (0: 2 unless the weight table is large)
    int window = 8;               // transitions per scheduling region
    bool diag = false;            // record s_memtime phase stamps (MDP_DIAG)
    bool xcd = true;              // XCD-aware block order
    bool qsum = true;             // Q rows come from k_qsum (else assembled from Pc in LDS)
    int slots = 8;                // registers caching transitions that recur (0: none)
};

// HIP source of `mdp_fwd_jit` for this plan; sets plan.epl when it was 0.
std::string mdp_jit_forward_source(MdpJitPlan &plan);

// Compile (or fetch from the memory / disk cache) a gfx950 code object.
// Returns 0 on success; on failure `log` holds the compiler output.
int mdp_jit_compile(const std::string &src, std::vector<char> &code, std::string &log);

#endif
