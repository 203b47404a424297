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


// ---- 3D (C4 / C5 inputs) -----------------------------------------------------
typedef struct csm_synth3d_config {
  uint64_t seed;
  double world_x, world_y, world_z;   // metres
  int32_t num_boxes;                  // pillars and crates
  int32_t num_nodes;
  int32_t num_submaps;
  int32_t scans_per_submap;           // nearest nodes inserted into each submap
  int32_t rings;                      // lidar rings
  int32_t azimuths;                   // returns per ring
  double min_elevation, max_elevation;  // radians
  double max_range;
  double range_noise;
  double high_resolution, low_resolution;  // HybridGrid resolutions
  double high_resolution_max_range;        // returns inserted into the high grid
  double high_voxel, low_voxel;            // adaptive voxel filter max_length
  double high_max_range;                   // node high-resolution cloud range
  int32_t high_min_points, low_min_points; // adaptive voxel filter min_num_points
  double low_max_range;
  int32_t histogram_size;
  double insert_voxel;                     // decimation of scans inserted into submaps
  int32_t threads;
  // Build only submaps [submap_begin, submap_begin + submap_count) of the
  // num_submaps-submap world (0 = all): a rank's shard, identical to those
  // submaps of the full world. Submap queries index the built range from 0.
  int32_t submap_begin, submap_count;
} csm_synth3d_config;

typedef struct csm_synth3d csm_synth3d;

void csm_synth3d_default_config(csm_synth3d_config* c);
int csm_synth3d_create(const csm_synth3d_config* cfg, csm_synth3d** out);
void csm_synth3d_destroy(csm_synth3d* w);
const double* csm_synth3d_node_poses(const csm_synth3d* w);  // x, y, z, yaw
const int32_t* csm_synth3d_submap_nodes(const csm_synth3d* w);
int64_t csm_synth3d_cloud(const csm_synth3d* w, int32_t node, int32_t kind, float* out,
                          int64_t capacity);
void csm_synth3d_node_histogram(const csm_synth3d* w, int32_t node, float* out);
void csm_synth3d_submap_histogram(const csm_synth3d* w, int32_t submap, float* out);
int64_t csm_synth3d_grid(const csm_synth3d* w, int32_t submap, int32_t grid, int32_t* ijk,
                         uint16_t* values, int64_t capacity);

#ifdef __cplusplus
}
#endif

#endif  // CSM_SYNTH_H_
