// Synthetic 2D world generator (bench / test inputs only; not the match path).
#ifndef CSM_SYNTH_H_
#define CSM_SYNTH_H_

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct csm_synth2d_config {
  uint64_t seed;
  double world_x, world_y;   // metres
  double resolution;         // metres per cell (grid and raster)
  int32_t num_nodes;
  int32_t num_submaps;
  int32_t submap_cells;      // submaps are submap_cells^2 cells
  int32_t beams;
  double fov;                // radians
  double max_range;          // metres
  double range_noise;        // sigma, metres
  int32_t decimate_to;       // 0 = keep every return
  double room_size;          // metres
  int32_t boxes_per_room;
  int32_t threads;           // 0 = min(16, hardware threads)
} csm_synth2d_config;

typedef struct csm_synth2d csm_synth2d;

void csm_synth2d_default_config(csm_synth2d_config* c);
int csm_synth2d_create(const csm_synth2d_config* cfg, csm_synth2d** out);
void csm_synth2d_destroy(csm_synth2d* w);
int32_t csm_synth2d_num_nodes(const csm_synth2d* w);
int32_t csm_synth2d_num_submaps(const csm_synth2d* w);
const int64_t* csm_synth2d_point_offsets(const csm_synth2d* w);
const float* csm_synth2d_points(const csm_synth2d* w);
const double* csm_synth2d_node_poses(const csm_synth2d* w);
const double* csm_synth2d_submap_max(const csm_synth2d* w);
const int32_t* csm_synth2d_submap_nodes(const csm_synth2d* w);
const uint16_t* csm_synth2d_submap_cells(const csm_synth2d* w);

#ifdef __cplusplus
}
#endif

#endif  // CSM_SYNTH_H_
