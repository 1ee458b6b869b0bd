// midaspom_amd/csrc/spom_jit.h -- problem-specialised forward kernel (hipRTC).
#ifndef SPOM_JIT_H
#define SPOM_JIT_H
#include <cstddef>
#include <cstdint>
#include <string>
#include <vector>

struct MdpJitPlan {
    std::vector<uint32_t> np;  // possible states per year
    uint32_t deg = 0;          // homogeneous transition degree D
    size_t ldR = 0;            // per-c coefficient block (doubles, stride RSP per use)
    int epl = 2;               // grid points per lane
    int window = 4;            // transitions per scheduling region
};

// HIP source of `mdp_fwd_jit` for this plan.
std::string mdp_jit_forward_source(const MdpJitPlan &plan);

// Compile (or fetch from the memory / disk cache) a gfx950 code object.
// Returns 0 on success; on failure `log` holds the compiler output.
int mdp_jit_compile(const std::string &src, std::vector<char> &code, std::string &log);

#endif
