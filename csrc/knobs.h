#pragma once
#include <cstdlib>

// Environment knob read ONCE per process and call site (A/B settings are fixed for a run; a
// getenv per conv call costs host time on every eager step -- ADVICE r4).  Knobs the tests
// toggle mid-process (P2P_CONV_VARIANT, P2P_NO_S2T, P2P_NO_HALO, P2P_S2T_GRID, P2P_S2T_F8) stay
// per-call reads at their sites and say so.
#define P2P_KNOB_ONCE(name) ([]() -> const char* { static const char* v_ = std::getenv(name); return v_; }())
