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

void sa_follow_matrix_host(double mh, double sg, double ta, double tb, double* out) {
  const SU2 m = sa_follow_matrix(mh, sg, ta, tb);
  out[0] = m.a.re, out[1] = m.a.im, out[2] = m.b.re, out[3] = m.b.im;
}

int sa_levels_count(void) { return kSALevels; }
}
