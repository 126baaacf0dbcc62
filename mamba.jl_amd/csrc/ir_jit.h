// ir_jit.h — host interface of the node-IR kernel specialisation (ir_jit.cpp).
#pragma once
#include <string>
#include <vector>

#include "../../include/mamba_hip.h"

// HIP source of the sweep kernel specialised for one lowered model: its node log densities and
// block term lists as straight-line code, `kinds` = bitmask of the scheme's sampler kinds,
// `dmax` = the widest AMM block (the unrolled factorization's step count).
std::string mmb_ir_jit_source(const mmb_model_spec& spec, const mmb_ir_model& ir, unsigned kinds, int dmax);

// Code object of `src` for gfx950: from the cache, else compiled by hipRTC and cached.
// Returns 0 on success; *info says which (or why it failed).
int mmb_ir_jit_obtain(const std::string& src, std::vector<char>* code, std::string* info);
