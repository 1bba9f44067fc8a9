// mpcb_kernels.h — host-visible launch interface of the HIP kernels (internal to the library).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "mpcb_model.h"

namespace mpcb {

constexpr int NX = 12;
constexpr int NU = 4;
constexpr int NZ = NX + NU;      // directions per instance = lanes per instance group
constexpr int GROUPS = 64 / NZ;  // instances per wavefront (4)
constexpr int NBOX_XTRA = 18;    // per-lane box-mode scratch values per stage (see solve kernel)

// Device-resident weights (row-major), uploaded once per handle.
template <class T>
struct Weights {
  T Q[NX * NX];
  T R[NU * NU];
  T QN[NX * NX];
  T lbu[NU], ubu[NU];
};

template <class T>
struct SolveArgs {
  int64_t B;
  int N;
  int mode;          // MPCB_MODE_ROLLOUT / MPCB_MODE_ITERATE
  int box;           // input boxes on
  int max_as_iter;
  T h;               // RK4 step
  T s;               // stage cost scaling
  Model<T> M;
  const Weights<T>* W;
  const T* x0; int64_t x0_sb;
  const T* xref; int64_t xref_sb;
  const T* uref; int64_t uref_sb;
  const T* wind; int64_t wind_sb;
  const T* xbar; const T* ubar;
  T* u0; T* X; T* U; int32_t* status;
  T* scratch;            // per-slot workspace
  int64_t slot_elems;    // elements per slot (one slot = one wavefront = GROUPS instances)
};

template <class T> hipError_t launch_solve(const SolveArgs<T>& a, int grid, hipStream_t st);
template <class T> int64_t solve_slot_elems(int N, int box);

template <class T>
hipError_t launch_linearize(int64_t B, int N, T h, const Model<T>& M, const T* xbar,
                            const T* ubar, const T* wind, int64_t wind_sb, T* A, T* Bm,
                            T* xnext, hipStream_t st);
template <class T>
hipError_t launch_sim_step(int64_t B, T h, const Model<T>& M, const T* x, const T* u,
                           const T* wind, int64_t wind_sb, T* xo, hipStream_t st);
template <class T>
hipError_t launch_gen_inputs(int64_t B, int N, T dt, uint64_t seed, uint64_t id_offset,
                             int ref_kind, T* x0, T* xref, int64_t xref_sb, T* uref,
                             int64_t uref_sb, T* wind, hipStream_t st);
template <class T>
hipError_t launch_histogram(int64_t B, int nu, const T* u0, double lo, double hi, int nbins,
                            unsigned long long* counts, hipStream_t st);

}  // namespace mpcb
