// Host-callable launchers of the kernels in csm_kernels.hip.
#ifndef CSM_LAUNCH_H_
#define CSM_LAUNCH_H_

#include <hip/hip_runtime.h>

#include "csm_device.h"

namespace csm {

hipError_t LaunchPyramidLevel0(const uint16_t* cells, const uint8_t* qtab, uint8_t* out, int n,
                               hipStream_t st);
hipError_t LaunchPyramidDouble(const uint8_t* prev, int pnx, int pny, uint8_t* next, int nnx,
                               int nny, int h, hipStream_t st);
hipError_t LaunchFast2dSearch(int grid, size_t dyn_lds, hipStream_t st, const SubmapDesc* submaps,
                              const PairDesc* pairs, const float* points, const float2* rot_table,
                              const WorkQueues& queues, unsigned long long* counters,
                              uint64_t* best, int32_t* status, unsigned long long* stats);
hipError_t LaunchPyramidQuad(const uint8_t* level, int wnx, int wny, int log_h, int km1,
                             uint32_t* out, int qw, int qh, int pws, int pph, int total,
                             hipStream_t st);
hipError_t LaunchFast2dSearchV2(int grid, size_t dyn_lds, hipStream_t st, const SubmapDesc* submaps,
                                const PairDesc* pairs, const float* points, const float2* rot_table,
                                const WorkQueues2& queues, unsigned long long* counters,
                                uint64_t* best, int32_t* status, unsigned long long* stats,
                                uint2* spill, int npad, int capc, bool hex, bool fifo,
                                uint64_t* best_hi, uint2* ties, int32_t* tie_count, bool collect);
hipError_t LaunchFast2dScoreQueries(int num_jobs, int npad, hipStream_t st, const SubmapDesc* submaps,
                                    const PairDesc* pairs, const float* points,
                                    const float2* rot_table, const ScoreJob* jobs,
                                    const int4* queries, int32_t* sums);
// Ordered walks to the reference's pick among tied maxima (ResolveTies):
// out[j] = (rot, x, y, found).
hipError_t LaunchFast2dWalk(int num_jobs, int npad, hipStream_t st, const SubmapDesc* submaps,
                            const PairDesc* pairs, const float* points, const float2* rot_table,
                            const WalkJob2* jobs, const int4* top, const int4* bounds, int4* out);
// ShrinkToFit bounds of (pair, rotation) jobs (ResolveTies).
hipError_t LaunchFast2dRotationBounds(int num_jobs, hipStream_t st, const SubmapDesc* submaps,
                                      const PairDesc* pairs, const float* points,
                                      const float2* rot_table, const int2* jobs, int4* bounds);
// Resident workgroups per CU of the v4/v5 search kernel at this dynamic LDS
// size (registers and LDS; 0 if the query fails).
int Fast2dSearchV2BlocksPerCu(bool hex, bool fifo, size_t dyn_lds);
// Widened level (into scratch, (wnx + km1) x (wny + km1) bytes), then its hex
// plane (total = 16-byte entries).
hipError_t LaunchPyramidHex(const uint8_t* level, int wnx, int wny, int log_h, int km1,
                            uint8_t* scratch, uint32_t* out, int qw, int qh, int pws, int pph,
                            int total, hipStream_t st);


hipError_t LaunchCellsToProbability(const uint16_t* cells, const float* ptab, float* out, int n,
                                    hipStream_t st);

}  // namespace csm

#endif  // CSM_LAUNCH_H_
