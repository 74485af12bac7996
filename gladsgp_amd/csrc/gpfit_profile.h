// Internal hooks of the optional event profiler (profile.hip); ids match GP_PROF_* in gpfit.h.
#pragma once
#include <hip/hip_runtime.h>

void gpfit_prof_begin(int id, hipStream_t st);
// begin of a pair that will bracket `launches` back-to-back launches of kernel `id`
void gpfit_prof_begin_n(int id, hipStream_t st, int launches);
void gpfit_prof_end(int id, hipStream_t st);
