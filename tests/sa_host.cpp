// Host build of the propagator's superadiabatic-frame device code (csrc/lzq_superadiabatic.h is
// __host__ __device__) for tests/test_superadiabatic_host.py: the exact functions the GPU kernels
// inline, checked on the CPU against the numpy restatement tests/lz_ref.py (TEST INFRASTRUCTURE).
#include "../baryon-and-dark-matter-densities-from-bounce--sourced-distributed-landau--zener-transport_amd/csrc/lzq_superadiabatic.h"

using namespace lzq;

extern "C" {

// the frame rotation of order kSALevels at Dh: out = (a.re, a.im, b.re, b.im)
void sa_frame_host(double Dh, double sg, double mh, double* out) {
  SU2 u;
  sa_levels_linear<kSALevels, true, false>(Dh, sg, mh, u, nullptr, nullptr);
  out[0] = u.a.re, out[1] = u.a.im, out[2] = u.b.re, out[3] = u.b.im;
}

// e_1 .. e_4 and g_0 .. g_3 (the phase nodes' levels)
void sa_levels4_host(double Dh, double sg, double mh, double* ev, double* gv) {
  SU2 u;
  sa_levels_linear<4, false, true>(Dh, sg, mh, u, ev, gv);
}

double sa_phase_host(double ta, double tb, double mh) { return sa_phase(ta, tb, mh); }

double sa_core_tau_host(double mh) { return sa_core_tau(mh); }

// both stretches of a cell: out = ML (4), MR (4)
void sa_cell_follow_host(double mh, double sg, double tl, double tr, double tau_c, int has_left, int has_right,
                         double* out) {
  for (int k = 0; k < 8; ++k) out[k] = (k % 4 == 0) ? 1.0 : 0.0;  // identity where a side is absent
  sa_cell_follow(mh, sg, tl, tr, tau_c, has_left != 0, has_right != 0, out);
}

int sa_levels_count(void) { return kSALevels; }
}
