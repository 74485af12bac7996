// Internal hooks of the optional event profiler (profile.hip); ids match GP_PROF_* in gpfit.h.
#pragma once
#include <hip/hip_runtime.h>

void gpfit_prof_begin(int id, hipStream_t st);
void gpfit_prof_end(int id, hipStream_t st);
