/*
 * csm_amd.h — C-ABI of the MI355X-native correlative scan matcher.
 *
 * Drop-in boundary for Cartographer's scan-matching hot path
 * (reference: juwangvsu/cartographer-1). Every entry point below replaces a
 * reference interface, cited as file:line relative to the reference root.
 * Plain pointers and sizes only; no C++ or torch types cross this boundary.
 *
 * Return codes: CSM_OK (0) = matched / success, CSM_NO_MATCH (1) = the search
 * completed without a score above min_score (the reference's `false` /
 * nullptr), negative = error. The reference aborts via glog CHECK on invariant
 * violations; the C++ shim (include/cartographer_amd/scan_matching.h) turns
 * negative codes into aborts to keep those semantics.
 *
 * Threading: matcher handles are re-entrant for concurrent match calls (the
 * reference calls const Match methods concurrently from ThreadPool workers,
 * constraint_builder_2d.cc:100-111). A single Match / MatchFullSubmap call
 * (csm_fast2d_match*, csm_fast3d_match*) takes a call context from a pool on
 * the matcher's context for its duration: its own HIP stream and scratch,
 * the matcher's device pyramid shared read-only, so concurrent callers'
 * searches overlap on the GPU. Calls that name a context (batches, RTCSM,
 * filters, refinement) serialise on that context's stream; use one context
 * per calling thread to run those concurrently. Destroying a handle while a
 * call uses it is the caller's error, as in the reference.
 */
#ifndef CSM_AMD_H_
#define CSM_AMD_H_

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define CSM_OK 0
#define CSM_NO_MATCH 1
#define CSM_EINVAL (-1)
#define CSM_EHIP (-2)
#define CSM_ENOMEM (-3)
#define CSM_ERANGE (-4) /* input exceeds the device path's index limits */

/* mapping/2d/map_limits.h:40-96 (resolution, max corner, CellLimits
 * xy_index.h:34-45). Cell (x, y) lives at flat index x + y * num_x_cells
 * (grid_2d.h:113-116); x counts down from max_y, y down from max_x
 * (map_limits.h:69-75). */
typedef struct csm_map_limits {
  double resolution;
  double max_x, max_y;
  int32_t num_x_cells, num_y_cells;
} csm_map_limits;

/* transform::Rigid2d (transform/rigid_transform.h:33-86): translation and an
 * unnormalized rotation angle. */
typedef struct csm_pose2d {
  double x, y, theta;
} csm_pose2d;

/* proto::FastCorrelativeScanMatcherOptions2D
 * (proto/scan_matching/fast_correlative_scan_matcher_options_2d.proto:19-30). */
typedef struct csm_fast2d_options {
  double linear_search_window;
  double angular_search_window;
  int32_t branch_and_bound_depth;
  /* Device-side search pyramid depth (>= branch_and_bound_depth, <= 12). The
   * branch and bound is exact, so extra coarse levels change only the work
   * done, never the result (DESIGN.md "Search"). 0 = automatic. */
  int32_t search_depth;
} csm_fast2d_options;

/* proto::RealTimeCorrelativeScanMatcherOptions
 * (proto/scan_matching/real_time_correlative_scan_matcher_options.proto:19-31). */
typedef struct csm_rt_options {
  double linear_search_window;
  double angular_search_window;
  double translation_delta_cost_weight;
  double rotation_delta_cost_weight;
} csm_rt_options;

typedef struct csm_context csm_context;   /* device, stream, scratch */
typedef struct csm_fast2d csm_fast2d;     /* one submap's device pyramid */
typedef struct csm_scan_set csm_scan_set; /* device-resident node clouds */

/* ---- context -------------------------------------------------------------- */
int csm_context_create(int32_t device, csm_context** out);
void csm_context_destroy(csm_context* ctx);
/* hipStream_t the context launches on (as void*), for event timing. */
void* csm_context_stream(csm_context* ctx);

/* Kernel timing, accumulated with HIP events on the context stream while
 * enabled: the candidate-scoring (search) kernel's total device milliseconds,
 * launches and algorithmic bytes (candidates scored x points x 1 B). */
typedef struct csm_timing {
  double search_kernel_ms;
  int64_t search_launches;
  double search_lookups;   /* candidates scored x points */
  double search_candidates;
  double other_kernel_ms;
  /* 3D: RTCSM3D scoring kernel time and lookups (candidates x points);
   * FastCSM3D search kernel time, launches and pyramid lookups. */
  double rt3d_kernel_ms;
  double rt3d_lookups;
  double fast3d_kernel_ms;
  int64_t fast3d_launches;
  double fast3d_lookups;
  /* Search health, accumulated while timing is enabled: pairs whose batch
   * search returned an error status (< 0), and the largest DFS stack depth
   * (entries) any workgroup reached (2D and 3D). */
  int64_t search_errors;
  int64_t stack_high_water;
  /* 2D searches whose maximum was reached by more than one leaf (the
   * reference's pick among them is restored, DESIGN.md §2 "Ties"), and those
   * of them picked by walking the reference's order on the device because
   * more than 4096 leaves tied (CSM_TIE_WALK; counted whether or not timing
   * is enabled). */
  int64_t tied_pairs;
  /* Named ties_unresolved before round 5 (same slot, same layout). */
  int64_t ties_walked;
  /* Pairs (2D and 3D) whose pick needed the whole lowest-resolution list
   * ordered (CSM_TIE_TOPLIST). 3D: pairs whose best sum was reached by more
   * than one leaf passing the low-resolution check, and those of them picked
   * by the ordered walk (more than 4096 such leaves). */
  int64_t ties_toplist;
  int64_t tied_pairs_3d;
  int64_t ties_walked_3d; /* named ties_unresolved_3d before round 5 */
} csm_timing;
void csm_context_enable_timing(csm_context* ctx, int32_t enable);
void csm_context_get_timing(csm_context* ctx, csm_timing* out);
void csm_context_reset_timing(csm_context* ctx);
/* Per pyramid level: candidates scored and scoring batches (v2 kernel),
 * accumulated while timing is enabled. Returns the number of levels written. */
int32_t csm_context_level_stats(csm_context* ctx, double* candidates, double* batches,
                                int32_t max_levels);

/* ---- FastCorrelativeScanMatcher2D ------------------------------------------
 * csm_fast2d_create replaces the constructor
 *   FastCorrelativeScanMatcher2D(const Grid2D&, const Options2D&)
 *   (fast_correlative_scan_matcher_2d.h:114-116, .cc:188-194)
 * and builds the PrecomputationGridStack2D (.cc:171-186) on the device.
 * `cells` are the grid's uint16 correspondence-cost values
 * (Grid2D::correspondence_cost_cells, grid_2d.h:97-99); min/max cc are
 * Grid2D::GetMin/MaxCorrespondenceCost (grid_2d.h:61-67). The cells are copied:
 * the caller may free them on return. */
int csm_fast2d_create(csm_context* ctx, const csm_map_limits* limits,
                      const uint16_t* cells, float min_correspondence_cost,
                      float max_correspondence_cost,
                      const csm_fast2d_options* options, csm_fast2d** out);
void csm_fast2d_destroy(csm_fast2d* m);

/* bool Match(const Rigid2d& initial_pose_estimate, const PointCloud&,
 *            float min_score, float* score, Rigid2d* pose_estimate) const
 *   (fast_correlative_scan_matcher_2d.h:127-129, .cc:198-208).
 * points: n x (x, y, z) floats (sensor::RangefinderPoint, point_cloud.h). */
int csm_fast2d_match(const csm_fast2d* m, const csm_pose2d* initial,
                     const float* points_xyz, int32_t n, float min_score,
                     float* score, csm_pose2d* pose);

/* bool MatchFullSubmap(const PointCloud&, float min_score, float* score,
 *                      Rigid2d* pose_estimate) const
 *   (fast_correlative_scan_matcher_2d.h:135-136, .cc:210-225). */
int csm_fast2d_match_full_submap(const csm_fast2d* m, const float* points_xyz,
                                 int32_t n, float min_score, float* score,
                                 csm_pose2d* pose);

/* Device bytes a matcher holds (its pyramid planes and cost grid), for a
 * caller's cache budget (the drop-in builders' matcher_cache_bytes; the
 * reference keeps every matcher until DeleteScanMatcher,
 * constraint_builder_2d.cc:165-186, :307-316). */
int64_t csm_fast2d_device_bytes(const csm_fast2d* m);

/* Test-visible: copies PrecomputationGrid2D level `level` (uint8 wide grid,
 * fast_correlative_scan_matcher_2d.h:49-93) to host. */
int csm_fast2d_read_level(const csm_fast2d* m, int32_t level, uint8_t* out,
                          int64_t capacity, int32_t* wide_nx, int32_t* wide_ny);

/* ---- Batched constraint search (the throughput path) ----------------------
 * Replaces the per-pair Tasks ConstraintBuilder2D schedules
 * (constraint_builder_2d.cc:77-137, ComputeConstraint :188-277): a set of
 * node clouds lives on the device once; each pair names a submap handle and a
 * node; results come back in pair order. */
int csm_scan_set_create(csm_context* ctx, const float* points_xyz,
                        const int64_t* offsets, int32_t num_scans,
                        csm_scan_set** out);
void csm_scan_set_destroy(csm_scan_set* s);
/* Appends num_scans clouds (offsets[0] == 0, as for create) to a live set:
 * the earlier scans keep their indices, device copies and cached rotation
 * tables, and the first new scan gets index *first_index. Lets a builder keep
 * one set across flushes (TrajectoryNode::Data clouds are immutable, so a
 * node's cloud is uploaded once, not once per flush). */
int csm_scan_set_append(csm_scan_set* s, const float* points_xyz,
                        const int64_t* offsets, int32_t num_scans,
                        int32_t* first_index);
/* Scans and points currently held (for a caller's cache limit). */
int csm_scan_set_size(const csm_scan_set* s, int32_t* num_scans, int64_t* num_points);

typedef struct csm_pair2d {
  int32_t submap;      /* index into the submaps[] array */
  int32_t scan;        /* index into the scan set */
  int32_t full_submap; /* 1 = MatchFullSubmap, 0 = Match(initial) */
  float min_score;
  csm_pose2d initial;  /* used when full_submap == 0 */
} csm_pair2d;

/* How a result was picked among exactly tied maxima (csm_result2d.tie;
 * DESIGN.md §2 "Exactly tied maxima"). The reference returns the first
 * maximal leaf its depth-first search visits
 * (fast_correlative_scan_matcher_2d.cc:276-312, :331-332, :344-376):
 *   NONE       one leaf reaches the maximum;
 *   ANCESTORS  several do, all under one highest-scoring lowest-resolution
 *              candidate: the pick follows the children's visiting order;
 *   TOPLIST    two distinct lowest-resolution candidates share the highest
 *              score: the pair's whole lowest-resolution list was scored and
 *              ordered with std::sort's introsort to find the first;
 *   WALK       more tied leaves than the collect pass records (4096): the
 *              device walks the reference's visiting order itself, from the
 *              sorted lowest-resolution list down to the first leaf at the
 *              maximum (any number of tied leaves).
 * Every branch returns the reference's leaf; none falls back to another. */
#define CSM_TIE_NONE 0
#define CSM_TIE_ANCESTORS 1
#define CSM_TIE_TOPLIST 2
#define CSM_TIE_WALK 3
/* Round-4 name of code 3 (before the walk resolved every such pair, it marked
 * them unresolved); kept so that callers written against it still compile. */
#define CSM_TIE_UNRESOLVED CSM_TIE_WALK

typedef struct csm_result2d {
  int32_t status;      /* CSM_OK, CSM_NO_MATCH or a negative error */
  float score;
  csm_pose2d pose;
  int32_t tie;         /* CSM_TIE_* (CSM_OK results only) */
  int32_t reserved;
} csm_result2d;

/* The submap handles may come from any context on ctx's device (e.g. one
 * whose stream builds the next batch's pyramids while ctx searches); the
 * scan set is ctx's. */
int csm_fast2d_match_batch(csm_context* ctx, csm_fast2d* const* submaps,
                           int32_t num_submaps, const csm_scan_set* scans,
                           const csm_pair2d* pairs, int64_t num_pairs,
                           csm_result2d* results);

/* ---- RealTimeCorrelativeScanMatcher2D --------------------------------------
 * double Match(const Rigid2d& initial_pose_estimate, const PointCloud&,
 *              const Grid2D&, Rigid2d* pose_estimate) const
 *   (real_time_correlative_scan_matcher_2d.h:66-68, .cc:117-149), for a
 * ProbabilityGrid. Returns CSM_OK and writes the best candidate's score. */
int csm_rt2d_match(csm_context* ctx, const csm_rt_options* options,
                   const csm_map_limits* limits, const uint16_t* cells,
                   float min_correspondence_cost, float max_correspondence_cost,
                   const csm_pose2d* initial, const float* points_xyz,
                   int32_t n, double* score, csm_pose2d* pose);

/* The same Match() for a TSDF2D grid (GridType::TSDF,
 * real_time_correlative_scan_matcher_2d.cc:38-59 and :162-167): the grid
 * crosses as its two uint16 arrays, correspondence_cost_cells() (TSD values,
 * tsdf_2d.cc:73-79) and weight_cells_ (tsdf_2d.cc:81-87), both x-fastest
 * num_x_cells * num_y_cells, plus the TSDValueConverter parameters
 * (truncation distance = max TSD, max weight; tsd_value_converter.cc:22-33).
 * Candidate score = sum((trunc - |tsd|) / trunc * weight) / sum(weight), 0 when
 * no point lands on a weighted cell; outside the limits a point reads
 * (-trunc, 0). */
int csm_rt2d_match_tsdf(csm_context* ctx, const csm_rt_options* options,
                        const csm_map_limits* limits, const uint16_t* tsd_cells,
                        const uint16_t* weight_cells, float truncation_distance,
                        float max_weight, const csm_pose2d* initial,
                        const float* points_xyz, int32_t n, double* score,
                        csm_pose2d* pose);

/* ---- correlative_scan_matcher_2d.h: search-space helpers ---------------------
 * The free functions and SearchParameters of correlative_scan_matcher_2d.h
 * (:35-68, .cc:27-127), host-side, with the reference's float/double
 * arithmetic (the device path computes the same values internally). */
typedef struct csm_linear_bounds {
  int32_t min_x, max_x, min_y, max_y;  /* inclusive pixel offsets */
} csm_linear_bounds;

typedef struct csm_search_parameters {
  int32_t num_angular_perturbations;
  double angular_perturbation_step_size;
  double resolution;
  int32_t num_scans;
  /* linear_bounds start as +-num_linear_perturbations for every scan. */
  int32_t num_linear_perturbations;
} csm_search_parameters;

/* SearchParameters(linear_search_window, angular_search_window, point_cloud,
 * resolution) (correlative_scan_matcher_2d.cc:27-52). */
int csm_search_parameters_init(double linear_search_window, double angular_search_window,
                               const float* points_xyz, int32_t n, double resolution,
                               csm_search_parameters* out);
/* SearchParameters(num_linear_perturbations, num_angular_perturbations,
 * angular_perturbation_step_size, resolution) — "for testing" (:54-66). */
int csm_search_parameters_init_for_testing(int32_t num_linear_perturbations,
                                           int32_t num_angular_perturbations,
                                           double angular_perturbation_step_size,
                                           double resolution, csm_search_parameters* out);
/* SearchParameters::ShrinkToFit (:68-91): bounds (num_scans entries) are
 * tightened in place against discrete scans (num_scans * points_per_scan
 * (x, y) cell indices, scan-major) and the grid's cell limits. */
int csm_search_parameters_shrink_to_fit(const csm_search_parameters* sp,
                                        const int32_t* discrete_xy, int32_t points_per_scan,
                                        int32_t num_x_cells, int32_t num_y_cells,
                                        csm_linear_bounds* bounds);
/* GenerateRotatedScans (:93-108): out_xyz holds num_scans * n points. */
int csm_generate_rotated_scans(const float* points_xyz, int32_t n,
                               const csm_search_parameters* sp, float* out_xyz);
/* DiscretizeScans (:110-127): num_scans rotated clouds of n points each
 * (scan-major), translated by (initial_x, initial_y) in float and turned
 * into cell indices by MapLimits::GetCellIndex; out_xy receives
 * num_scans * n (x, y) pairs. */
int csm_discretize_scans(const csm_map_limits* limits, const float* rotated_xyz, int32_t n,
                         int32_t num_scans, float initial_x, float initial_y, int32_t* out_xy);

/* Candidate2D (correlative_scan_matcher_2d.h:71-98): score is filled in by
 * ScoreCandidates. */
typedef struct csm_candidate2d {
  int32_t scan_index, x_index_offset, y_index_offset;
  float score;
} csm_candidate2d;

/* RealTimeCorrelativeScanMatcher2D::ScoreCandidates(grid, discrete_scans,
 * search_parameters, candidates*) (real_time_correlative_scan_matcher_2d.h:
 * 75-78, .cc:151-176; visible for testing): every candidate's score =
 * mean probability of its discrete scan shifted by its offsets, times
 * exp(-(hypot(x, y) * w_t + |orientation| * w_r)^2) with the candidate's
 * x, y, orientation from the search parameters. discrete_xy as
 * csm_discretize_scans writes it. */
int csm_rt2d_score_candidates(csm_context* ctx, const csm_rt_options* options,
                              const csm_map_limits* limits, const uint16_t* cells,
                              float min_correspondence_cost, float max_correspondence_cost,
                              const int32_t* discrete_xy, int32_t num_scans,
                              int32_t points_per_scan, const csm_search_parameters* sp,
                              csm_candidate2d* candidates, int64_t num_candidates);
/* The same over a TSDF2D (grid arrays as csm_rt2d_match_tsdf). */
int csm_rt2d_score_candidates_tsdf(csm_context* ctx, const csm_rt_options* options,
                                   const csm_map_limits* limits, const uint16_t* tsd_cells,
                                   const uint16_t* weight_cells, float truncation_distance,
                                   float max_weight, const int32_t* discrete_xy,
                                   int32_t num_scans, int32_t points_per_scan,
                                   const csm_search_parameters* sp,
                                   csm_candidate2d* candidates, int64_t num_candidates);

/* ---- 3D: HybridGrid ----------------------------------------------------------
 * A HybridGrid (mapping/3d/hybrid_grid.h:463-545) crosses the boundary as the
 * list its iterator / ToProto yields (hybrid_grid.h:530-541): cell indices
 * (x, y, z) and uint16 probability values. The device keeps a dense brick
 * over the known cells' bounding box; outside it the value is 0 (unknown,
 * probability kMinProbability), as DynamicGrid::value returns for cells never
 * set (:260-279). `grid_size` is DynamicGrid::grid_size() of the source grid
 * (FastCorrelativeScanMatcher3D's width_in_voxels, .cc:120); 0 = derive it from
 * the indices with DynamicGrid's growth rule (128 << k, indices in
 * [-size/2, size/2)). The cells are copied. */
typedef struct csm_hybrid_grid csm_hybrid_grid;
int csm_hybrid_grid_create(csm_context* ctx, float resolution, const int32_t* xyz_indices,
                           const uint16_t* values, int64_t count, int32_t grid_size,
                           csm_hybrid_grid** out);
/* `num` grids in one call, each as csm_hybrid_grid_create builds it (the
 * same bricks and values), with one upload and one launch per build step for
 * all of them: for a caller that builds many submaps' grids at once (the
 * constraint builder's matcher construction, constraint_builder_3d.cc:
 * 170-198). grid_sizes may be NULL (every grid derives its size). */
int csm_hybrid_grid_create_batch(csm_context* ctx, int32_t num, const float* resolutions,
                                 const int32_t* const* xyz_indices, const uint16_t* const* values,
                                 const int64_t* counts, const int32_t* grid_sizes,
                                 csm_hybrid_grid** out);
void csm_hybrid_grid_destroy(csm_hybrid_grid* g);
/* Bounding box origin / extent of the device brick and the grid size. */
int csm_hybrid_grid_info(const csm_hybrid_grid* g, int32_t* origin3, int32_t* dims3,
                         int32_t* grid_size);
/* Test-visible lookups on the device grid, with the kernels' own code:
 * HybridGrid::GetProbability at n cell indices (hybrid_grid.h:496-499; unknown
 * cells give kMinProbability), and InterpolatedProbabilityGrid::
 * GetInterpolatedValue at n points (interpolated_grid.h:48-105, the
 * CeresScanMatcher3D cost's interpolation). */
int csm_hybrid_grid_get_probability(const csm_hybrid_grid* g, const int32_t* xyz_indices, int64_t n,
                                    float* out);
int csm_hybrid_grid_interpolate(const csm_hybrid_grid* g, const double* xyz, int64_t n,
                                double* out);

/* transform::Rigid3d: translation and rotation quaternion (w, x, y, z). */
typedef struct csm_pose3d {
  double t[3];
  double q[4];
} csm_pose3d;

/* ---- RealTimeCorrelativeScanMatcher3D ----------------------------------------
 * float Match(const Rigid3d& initial_pose_estimate, const PointCloud&,
 *             const HybridGrid&, Rigid3d* pose_estimate) const
 *   (real_time_correlative_scan_matcher_3d.h:47-50, .cc:34-54). */
int csm_rt3d_match(csm_context* ctx, const csm_rt_options* options, const csm_hybrid_grid* grid,
                   const csm_pose3d* initial, const float* points_xyz, int32_t n, float* score,
                   csm_pose3d* pose);

/* The search window Match uses (GenerateExhaustiveSearchTransforms, :55-95):
 * (2L+1)^3 translations and (2A+1)^3 rotations for this cloud and grid
 * resolution. Candidate index = t * num_rotations + r. */
int csm_rt3d_window(const csm_rt_options* options, float resolution, const float* points_xyz,
                    int32_t n, int32_t* num_translations, int32_t* num_rotations);

/* Test-visible: ScoreCandidate (:97-113, score after the exp penalty) of
 * every translation for each of `num_rotations` rotation indices of the
 * window, computed by the same kernel as Match; scores[k * num_translations
 * + t] for rotations[k]. */
int csm_rt3d_score_rotations(csm_context* ctx, const csm_rt_options* options,
                             const csm_hybrid_grid* grid, const csm_pose3d* initial,
                             const float* points_xyz, int32_t n, const int32_t* rotations,
                             int32_t num_rotations, float* scores);

/* ---- FastCorrelativeScanMatcher3D --------------------------------------------
 * proto::FastCorrelativeScanMatcherOptions3D
 * (proto/scan_matching/fast_correlative_scan_matcher_options_3d.proto). */
typedef struct csm_fast3d_options {
  int32_t branch_and_bound_depth;
  int32_t full_resolution_depth;
  double min_rotational_score;
  double min_low_resolution_score;
  double linear_xy_search_window;
  double linear_z_search_window;
  double angular_search_window;
} csm_fast3d_options;

typedef struct csm_fast3d csm_fast3d;

/* FastCorrelativeScanMatcher3D(const HybridGrid&, const HybridGrid* low_res,
 *   const Eigen::VectorXf* histogram, const Options3D&)
 *   (fast_correlative_scan_matcher_3d.h:75-79, .cc:112-123). The pyramid
 * (PrecomputationGridStack3D, .cc:57-77) is built on the device from
 * `high_resolution`; the histogram is copied. As in the reference (which keeps
 * raw pointers, .h:149-150) `low_resolution` must outlive the matcher. */
int csm_fast3d_create(csm_context* ctx, const csm_hybrid_grid* high_resolution,
                      const csm_hybrid_grid* low_resolution, const float* histogram,
                      int32_t histogram_size, const csm_fast3d_options* options,
                      csm_fast3d** out);
/* `count` FastCorrelativeScanMatcher3D constructions in one call (a sweep
 * that builds many submaps' matchers at once, e.g. ConstraintBuilder3D's
 * DispatchScanMatcherConstruction for every submap of a loaded map,
 * constraint_builder_3d.cc:170-198): out[i] is what csm_fast3d_create(ctx,
 * high[i], low[i], histograms[i], histogram_sizes[i], options) returns, with
 * each pyramid level built for all of them in one launch. On error no
 * matcher is returned. count <= 65535. */
int csm_fast3d_create_batch(csm_context* ctx, int32_t count,
                            const csm_hybrid_grid* const* high_resolution,
                            const csm_hybrid_grid* const* low_resolution,
                            const float* const* histograms, const int32_t* histogram_sizes,
                            const csm_fast3d_options* options, csm_fast3d** out);
void csm_fast3d_destroy(csm_fast3d* m);
/* Device bytes of the matcher's pyramid (levels and octet planes), and of a
 * HybridGrid's bricks (as csm_fast2d_device_bytes). */
int64_t csm_fast3d_device_bytes(const csm_fast3d* m);
int64_t csm_hybrid_grid_device_bytes(const csm_hybrid_grid* g);
/* Test-visible: copies pyramid level `level` (dense brick, x fastest). */
int csm_fast3d_read_level(const csm_fast3d* m, int32_t level, uint8_t* out, int64_t capacity,
                          int32_t* origin3, int32_t* dims3);

/* The parts of TrajectoryNode::Data the matcher reads (trajectory_node.h):
 * high/low resolution point clouds, the rotational histogram and the
 * gravity alignment (w, x, y, z). */
typedef struct csm_node3d {
  const float* high_resolution_xyz;
  int32_t num_high_resolution;
  const float* low_resolution_xyz;
  int32_t num_low_resolution;
  const float* histogram;
  int32_t histogram_size;
  double gravity_alignment[4];
} csm_node3d;

/* FastCorrelativeScanMatcher3D::Result (fast_correlative_scan_matcher_3d.h:68-73). */
typedef struct csm_result3d {
  int32_t status; /* CSM_OK, CSM_NO_MATCH (the reference's nullptr) or error */
  float score;
  csm_pose3d pose;
  float rotational_score;
  float low_resolution_score;
  int32_t tie;    /* CSM_TIE_*: how the pick among exactly tied leaves was made */
  int32_t reserved;
} csm_result3d;

/* std::unique_ptr<Result> Match(const Rigid3d& global_node_pose,
 *   const Rigid3d& global_submap_pose, const TrajectoryNode::Data&, float min_score)
 *   (fast_correlative_scan_matcher_3d.h:89-92, .cc:127-143). */
int csm_fast3d_match(const csm_fast3d* m, const csm_pose3d* global_node_pose,
                     const csm_pose3d* global_submap_pose, const csm_node3d* node,
                     float min_score, csm_result3d* result);
/* std::unique_ptr<Result> MatchFullSubmap(const Quaterniond& global_node_rotation,
 *   const Quaterniond& global_submap_rotation, const TrajectoryNode::Data&, float)
 *   (fast_correlative_scan_matcher_3d.h:98-101, .cc:145-170). Rotations (w,x,y,z). */
int csm_fast3d_match_full_submap(const csm_fast3d* m, const double* global_node_rotation,
                                 const double* global_submap_rotation, const csm_node3d* node,
                                 float min_score, csm_result3d* result);

/* Batched 3D constraint search (ConstraintBuilder3D tasks,
 * constraint_builder_3d.cc:200-305): results in pair order. For full_submap
 * pairs only the rotations of the two poses are used. */
typedef struct csm_pair3d {
  int32_t submap;
  int32_t node;
  int32_t full_submap;
  float min_score;
  csm_pose3d node_pose;
  csm_pose3d submap_pose;
} csm_pair3d;

int csm_fast3d_match_batch(csm_context* ctx, csm_fast3d* const* submaps, int32_t num_submaps,
                           const csm_node3d* nodes, int32_t num_nodes, const csm_pair3d* pairs,
                           int64_t num_pairs, csm_result3d* results);

/* ---- CeresScanMatcher2D refinement ------------------------------------------
 * ConstraintBuilder2D::ComputeConstraint refines every accepted match with
 * CeresScanMatcher2D::Match(target_translation = match translation,
 * initial = match, filtered cloud, submap grid) (constraint_builder_2d.cc:
 * 245-249; ceres_scan_matcher_2d.cc:64-105). csm_ceres2d_refine_batch runs
 * that refinement for n (submap, scan) items on the device, over the submaps'
 * csm_fast2d handles (their correspondence-cost grids) and a scan set.
 * Ceres is not part of this library: the solver restates Ceres 1.13's
 * trust-region Levenberg-Marquardt (the version scripts/install_ceres.sh:20
 * pins), pinned by the reference's ceres_scan_matcher_2d_test.cc.
 * iterations (may be NULL) receives the iterations each item ran. */
typedef struct csm_ceres2d_options {
  /* proto::CeresScanMatcherOptions2D (pose_graph.lua:30-39 defaults 20, 10, 1;
   * ceres_solver_options.max_num_iterations = 10). */
  double occupied_space_weight;
  double translation_weight;
  double rotation_weight;
  int32_t max_num_iterations;
  /* ceres_solver_options.use_nonmonotonic_steps (pose_graph.lua:35: true). */
  int32_t use_nonmonotonic_steps;
} csm_ceres2d_options;

typedef struct csm_refine2d {
  int32_t submap;  /* index into submaps[] */
  int32_t scan;    /* index into the scan set */
  csm_pose2d initial;
  double target_x, target_y;
} csm_refine2d;

int csm_ceres2d_refine_batch(csm_context* ctx, csm_fast2d* const* submaps, int32_t num_submaps,
                             const csm_scan_set* scans, const csm_refine2d* items, int64_t n,
                             const csm_ceres2d_options* options, csm_pose2d* out,
                             int32_t* iterations);

/* CeresScanMatcher3D refinement (ConstraintBuilder3D::ComputeConstraint,
 * constraint_builder_3d.cc:264-275; ceres_scan_matcher_3d.cc:84-160): the
 * match pose is refined against the submap's high- and low-resolution
 * HybridGrids with the node's high- and low-resolution clouds. Item i uses
 * grids[high_grid], grids[low_grid] and nodes[node]; target is the match
 * translation. Same solver notes as csm_ceres2d_refine_batch. */
typedef struct csm_ceres3d_options {
  /* proto::CeresScanMatcherOptions3D (pose_graph.lua:49-60: 5, 30, 10, 1,
   * max_num_iterations 10). */
  double occupied_space_weight_0;
  double occupied_space_weight_1;
  double translation_weight;
  double rotation_weight;
  int32_t max_num_iterations;
  /* ceres_solver_options.use_nonmonotonic_steps (pose_graph.lua:56: false). */
  int32_t use_nonmonotonic_steps;
} csm_ceres3d_options;

typedef struct csm_refine3d {
  int32_t high_grid, low_grid, node;
  csm_pose3d initial;
  double target[3];
} csm_refine3d;

/* The grids may come from any context on ctx's device; the refinement waits
 * on the device for their builds. */
int csm_ceres3d_refine_batch(csm_context* ctx, const csm_hybrid_grid* const* grids,
                             int32_t num_grids, const csm_node3d* nodes, int32_t num_nodes,
                             const csm_refine3d* items, int64_t n,
                             const csm_ceres3d_options* options, csm_pose3d* out,
                             int32_t* iterations);

/* ---- submap grid formats ---------------------------------------------------
 * Submap2D::Finish (submap_2d.cc:146-150) crops a finished submap's grid to
 * its known cells: ProbabilityGrid::ComputeCroppedGrid
 * (probability_grid.cc:91-106) with Grid2D::ComputeCroppedLimits
 * (grid_2d.cc:110-120). `cells` are num_x_cells * num_y_cells uint16 values
 * (x fastest); the known box is the bounding box of the nonzero cells.
 * csm_grid2d_cropped_limits returns the cropped MapLimits and the offset
 * (x, y) of its first cell; csm_grid2d_crop also copies the cells into
 * cropped_cells (capacity >= cropped nx * ny). An all-unknown grid crops to
 * one unknown cell, as the reference does. Host-only. */
int csm_grid2d_cropped_limits(const csm_map_limits* limits, const uint16_t* cells,
                              int32_t* offset_xy, csm_map_limits* cropped);
int csm_grid2d_crop(const csm_map_limits* limits, const uint16_t* cells,
                    csm_map_limits* cropped, uint16_t* cropped_cells, int64_t capacity);

/* ---- node clouds: voxel filters -------------------------------------------
 * sensor::VoxelFilter and sensor::AdaptiveVoxelFilter
 * (sensor/internal/voxel_filter.h, voxel_filter.cc:212-232 and :263-268), the
 * filters that make the clouds the matchers search with
 * (local_trajectory_builder_2d.cc:61-62, :229-231;
 * local_trajectory_builder_3d.cc:682-683, :735-748). A batch of clouds: cloud
 * c is points [offsets[c], offsets[c+1]) of xyz (float x, y, z). keep[i] = 1
 * when point i survives; the reference returns the survivors in input order
 * and filters intensities with the same mask. counts[c] = survivors of cloud c
 * (may be NULL). The kept set is the reference's exactly (same voxel keys, same
 * minstd_rand0 reservoir draws). Clouds of up to 8192 points (larger:
 * CSM_ERANGE). */
typedef struct csm_adaptive_voxel_filter_options {
  /* proto::AdaptiveVoxelFilterOptions
   * (sensor/proto/adaptive_voxel_filter_options.proto): all floats. */
  float max_length;
  float min_num_points;
  float max_range;
} csm_adaptive_voxel_filter_options;

int csm_voxel_filter(csm_context* ctx, const float* xyz, const int64_t* offsets,
                     int32_t num_clouds, float resolution, uint8_t* keep, int32_t* counts);
int csm_adaptive_voxel_filter(csm_context* ctx, const float* xyz, const int64_t* offsets,
                              int32_t num_clouds, const csm_adaptive_voxel_filter_options* options,
                              uint8_t* keep, int32_t* counts);
/* The same on device-resident buffers (d_offsets relative to d_xyz), enqueued
 * on the context's stream without synchronising; max_points bounds every
 * cloud's size. */
int csm_voxel_filter_device(csm_context* ctx, const float* d_xyz, const int64_t* d_offsets,
                            int32_t num_clouds, int32_t max_points, float resolution,
                            uint8_t* d_keep, int32_t* d_counts);
int csm_adaptive_voxel_filter_device(csm_context* ctx, const float* d_xyz,
                                     const int64_t* d_offsets, int32_t num_clouds,
                                     int32_t max_points,
                                     const csm_adaptive_voxel_filter_options* options,
                                     uint8_t* d_keep, int32_t* d_counts);

/* ---- pbstream ingest --------------------------------------------------------
 * Reads a serialized state file (io/proto_stream.cc:26-86: magic, then per
 * message an 8-byte size and a gzip member; SerializationHeader then
 * SerializedData, mapping/proto/serialization.proto:72-88) and keeps what a
 * ConstraintBuilder2D needs: every Submap2D (id, local pose, finished flag,
 * Grid2D as in Grid2D::Grid2D(proto), mapping/2d/grid_2d.cc:75-96) and every
 * Node (id, timestamp, gravity alignment, local pose and the decompressed
 * filtered_gravity_aligned_point_cloud, sensor/compressed_point_cloud.cc:79-97).
 * Poses are (tx, ty, tz, qw, qx, qy, qz); gravity_alignment is (w, x, y, z).
 * 3D submaps and the nodes' 3D clouds are kept too (below). Other message
 * kinds (pose graph, options, sensor data) are skipped. Host-only; returns CSM_EINVAL for a malformed file. Pass NULL for
 * any output not wanted; cells / xyz need capacity >= the item's size
 * (CSM_ERANGE otherwise). */
typedef struct csm_pbstream csm_pbstream;
int csm_pbstream_open(const char* path, csm_pbstream** out);
void csm_pbstream_close(csm_pbstream* stream);
uint32_t csm_pbstream_format_version(const csm_pbstream* stream);
int32_t csm_pbstream_num_submaps2d(const csm_pbstream* stream);
int32_t csm_pbstream_num_nodes(const csm_pbstream* stream);
/* ids = (trajectory_id, submap_index); min_max_cc = (min, max)
 * correspondence cost; cells are num_x_cells * num_y_cells values, x fastest. */
int csm_pbstream_submap2d(const csm_pbstream* stream, int32_t index, int32_t* ids,
                          csm_map_limits* limits, float* min_max_cc, int32_t* finished,
                          double* local_pose7, uint16_t* cells, int64_t capacity);
/* ids = (trajectory_id, node_index); capacity and num_points count points. */
int csm_pbstream_node(const csm_pbstream* stream, int32_t index, int32_t* ids,
                      int64_t* timestamp, double* local_pose7, double* gravity_alignment,
                      float* xyz, int64_t capacity, int32_t* num_points);
/* A node's clouds: which = 0 filtered_gravity_aligned_point_cloud (what
 * csm_pbstream_node returns), 1 high_resolution_point_cloud, 2
 * low_resolution_point_cloud (the 3D matcher's inputs); and its
 * rotational_scan_matcher_histogram (size = number of buckets). */
int csm_pbstream_node_cloud(const csm_pbstream* stream, int32_t index, int32_t which, float* xyz,
                            int64_t capacity, int32_t* num_points);
int csm_pbstream_node_histogram(const csm_pbstream* stream, int32_t index, float* histogram,
                                int32_t capacity, int32_t* size);
/* Submap3D (submap.proto:32-39): ids, finished, local pose, the cell counts of
 * its (high, low) resolution HybridGrids and its histogram size. A grid's
 * cells come back as csm_hybrid_grid_create takes them (xyz_indices 3 per
 * cell, uint16 values as HybridGrid(proto) stores them, hybrid_grid.h:473-484);
 * which = 0 high, 1 low resolution. */
int32_t csm_pbstream_num_submaps3d(const csm_pbstream* stream);
int csm_pbstream_submap3d(const csm_pbstream* stream, int32_t index, int32_t* ids,
                          int32_t* finished, double* local_pose7, int64_t* num_cells,
                          int32_t* histogram_size);
int csm_pbstream_submap3d_grid(const csm_pbstream* stream, int32_t index, int32_t which,
                               float* resolution, int32_t* xyz_indices, uint16_t* values,
                               int64_t capacity);
int csm_pbstream_submap3d_histogram(const csm_pbstream* stream, int32_t index, float* histogram,
                                    int32_t capacity);

/* ---- Multi-GPU hand-off ------------------------------------
 * The constraint queue shards across ranks (one process per GPU) with no
 * data-path collective; the one exchange is gathering every rank's accepted
 * constraints to rank 0 for the CPU pose-graph solve, where WhenDone's
 * submission order is restored (constraint_builder_2d.cc:279-300 delivers
 * results in submission order through one callback). The reference runs one
 * process and has no counterpart; these calls are what a sharded
 * ConstraintBuilder2D (include/cartographer_amd/constraint_builder_2d.h,
 * set_communicator) uses. Transports: RCCL over xGMI (rank r on its context's
 * device; rank 0 makes the id with csm_comm_get_unique_id and the caller
 * distributes it) or TCP between host processes (CPU tests, rehearsals). */
#define CSM_COMM_ID_BYTES 128
#define CSM_REDUCE_SUM 0
#define CSM_REDUCE_MAX 1
typedef struct csm_comm csm_comm;
int csm_comm_get_unique_id(uint8_t* id /* CSM_COMM_ID_BYTES */);
int csm_comm_create_rccl(csm_context* ctx, int32_t rank, int32_t world_size, const uint8_t* id,
                         csm_comm** out);
/* Rank 0 listens on `port`; the others connect to root_host:port. */
int csm_comm_create_tcp(int32_t rank, int32_t world_size, const char* root_host, int32_t port,
                        csm_comm** out);
void csm_comm_destroy(csm_comm* comm);
int32_t csm_comm_rank(const csm_comm* comm);
int32_t csm_comm_size(const csm_comm* comm);
/* Collective: every rank contributes send_bytes; rank 0 keeps all blobs in
 * rank order (total in *total_bytes, 0 on other ranks) and copies them out
 * with csm_comm_gathered (sizes: world_size entries, bytes per rank). */
int csm_comm_gather(csm_comm* comm, const void* send, int64_t send_bytes, int64_t* total_bytes);
int csm_comm_gathered(const csm_comm* comm, void* out, int64_t capacity, int64_t* sizes);
/* Collective: element-wise sum or max over ranks, in place. */
int csm_comm_allreduce_i64(csm_comm* comm, int64_t* values, int32_t count, int32_t op);
int csm_comm_barrier(csm_comm* comm);
/* Dynamic work claiming: the shared queue of the reference's
 * common::ThreadPool (thread_pool.cc:80-106, idle workers take the next task;
 * ConstraintBuilder2D schedules one task per pair, constraint_builder_2d.cc:102-111)
 * stretched over ranks. claim_open is collective: rank 0 serves a table of
 * int64 counters from a host thread on `port`, the others connect to
 * root_host:port (any transport; a world of 1 keeps the table locally).
 * fetch_add is NOT collective: *old_value = counter[key], counter[key] += delta,
 * atomically across ranks; counters start at 0. */
int csm_comm_claim_open(csm_comm* comm, const char* root_host, int32_t port);
int csm_comm_fetch_add(csm_comm* comm, int64_t key, int64_t delta, int64_t* old_value);

/* Human-readable text for a return code. */
const char* csm_strerror(int code);

#ifdef __cplusplus
}
#endif

#endif /* CSM_AMD_H_ */
