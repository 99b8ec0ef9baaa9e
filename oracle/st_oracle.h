/*
 * st_oracle.h -- CPU restatement of the reference's hot path (TEST INFRASTRUCTURE).
 *
 * This library is the parity CHECKER for the MI355X product under
 * splat-transform_amd/.  Only tests/, __graft_entry__.smoke() and bench.py's
 * cpu_baseline leg may load it; the product never links or calls it.
 *
 * Every function restates one reference function (file:line into
 * /root/reference/src) with JS-number (IEEE f64) semantics, evaluation order
 * preserved, compiled with -ffp-contract=off.  It is pinned against the
 * golden vectors in tests/golden/ produced by running the reference's own
 * modules (see tests/golden/README.md).
 */
#ifndef ST_ORACLE_H
#define ST_ORACLE_H
#include <stdint.h>
#ifdef __cplusplus
extern "C" {
#endif

/* V8 Math.exp / Math.log are fdlibm ports (ieee754::exp / ieee754::log). */
double st_o_exp(double x);
double st_o_log(double x);

/* PlayCanvas 2.11.8 math restated (process.ts:75-79, transform.ts:13-14). */
void st_o_quat_from_euler(double ex, double ey, double ez, double q_xyzw[4]);
void st_o_mat4_trs(const double t[3], const double q_xyzw[4], double s, float m[16]);
void st_o_mat3_from_quat(const double q_xyzw[4], float m[9]);
/* RotateSH constructor (rotate-sh.ts:49-149): band matrices, row-major. */
void st_o_rotate_sh(const float m3[9], double sh1[9], double sh2[25], double sh3[49]);

/* transform() (transform.ts:12-65), in place.  Any group pointer may be NULL
 * when the table lacks those columns; sh has sh_coeffs*3 channel-major
 * columns (f_rest_{k + ch*C}). */
void st_o_transform(uint64_t n, float *x, float *y, float *z, float *const rot[4],
                    float *const scale[3], float *const *sh, int sh_coeffs,
                    const float m4[16], const double r_xyzw[4], double s,
                    const double sh1[9], const double sh2[25], const double sh3[49]);

/* filterNaN predicate + stable compaction (process.ts:47-61,84-95). */
uint64_t st_o_filter_finite(uint64_t n, int ncol, const float *const *cols, uint32_t *out_idx);

/* generateOrdering (ordering.ts:4-110), indices permuted in place. */
void st_o_morton_order(const float *x, const float *y, const float *z, uint32_t *indices, uint64_t n);

/* writeCompressedPly body (write-compressed-ply.ts:56-109) + CompressedChunk.pack
 * (compressed-chunk.ts:44-180).  m14 = the 14 CompressedChunk.members columns
 * in order x,y,z,scale_0..2,f_dc_0..2,opacity,rot_0..3.  `order` is the
 * Morton permutation.  chunk: ceil(n/256)*18 f32; vertex: n*4 u32; sh_out: n*nsh. */
void st_o_pack_compressed(uint64_t n, const float *const m14[14], const float *const *sh, int nsh,
                          const uint32_t *order, float *chunk, uint32_t *vertex, uint8_t *sh_out);

/* kmeans (k-means.ts:137-201) on the --no-gpu path (kd-tree assign).
 * cols: d columns of n points.  draws: the Math.random stream.  centroids:
 * d columns of k (or n when n < k).  Returns 0, or -1 on a reference crash
 * condition (non-finite distance), -2 draws exhausted. */
/* OpenMP threads for st_o_kmeans's assign (labels unchanged; default 1) */
void st_o_set_threads(int threads);
int st_o_kmeans(const float *const *cols, int d, uint64_t n, int k, int iters,
                const double *draws, uint64_t ndraws, uint64_t *used,
                float *centroids, uint32_t *labels);

/* One clusterKdTreeCpu pass (k-means.ts:103-121): KdTree over the given
 * centroids (d columns of k) + findNearest for every point.  Used to time
 * the CPU baseline of the assign step. */
int st_o_kmeans_assign(const float *const *cols, int d, uint64_t n, const float *centroids, int k, uint32_t *labels);
int st_o_kmeans_assign_mt(const float *const *cols, int d, uint64_t n, const float *centroids, int k,
                          uint32_t *labels, int threads);

/* cluster1d (write-sog.ts:56-99): centroids[256] sorted ascending, labels u8 (ncols x n). */
int st_o_cluster1d(const float *const *cols, int ncols, uint64_t n, int iters,
                   const double *draws, uint64_t ndraws, uint64_t *used,
                   float *centroids, uint8_t *labels);

/* writeSog texture + meta generation (write-sog.ts:110-370), identity layout. */
typedef struct {
    int width, height;
    double means_min[3], means_max[3];
    float scales_codebook[256];
    float sh0_codebook[256];
    int sh_bands, palette_size;
    float shn_codebook[256];
    int shn_width, shn_height;
} st_o_sog_meta;

/* cols: the 14 members (as st_o_pack_compressed) ; sh as above.
 * means_l, means_u, quats, scales, sh0, shn_labels: width*height*4 each;
 * shn_centroids: (64*C) * ceil(K/64) * 4. */
int st_o_sog(uint64_t n, const float *const m14[14], const float *const *sh, int sh_coeffs, int iters,
             const double *draws, uint64_t ndraws, uint64_t *used, st_o_sog_meta *meta,
             uint8_t *means_l, uint8_t *means_u, uint8_t *quats, uint8_t *scales, uint8_t *sh0,
             uint8_t *shn_centroids, uint8_t *shn_labels);

/* compressed-PLY reader (decompress-ply.ts:82-232): see st_oracle.c */
void st_o_decompress_ply(uint64_t n, const float *const chunk[18], const uint32_t *const vertex[4],
                         const uint8_t *const *sh, int nsh, float *const *out);

#ifdef __cplusplus
}
#endif
#endif
