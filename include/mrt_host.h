/*
 * mrt_host.h — C-ABI of the host side around the hot path: scenes, the SBVH
 * builder, the Compact2 layout and its bvhcache .dat format, the camera and
 * ray generation. These are the producers of the trace kernel's inputs
 * (SURVEY.md §8f "next" rows), restating:
 *   src/rt/Scene.cc:35-101, src/framework/io/MeshWavefrontIO.cc:258-467   (scene, OBJ)
 *   src/rt/bvh/SplitBVHBuilder.cc:55-485, src/framework/base/Sort.cc:63-239 (SBVH)
 *   src/rt/cuda/CudaBVH.cc:79-116,270-380, Renderer.cc:157-217            (Compact2, cache)
 *   src/rt/ray/RayGen.cc:50-142, RayGenKernels.cu:79-227, PixelTable.cc    (ray generation)
 * All buffers here are HOST memory. Functions return 0 or an MRTH_ERR_* code.
 */
#ifndef MRT_HOST_H
#define MRT_HOST_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

enum { MRTH_OK = 0, MRTH_ERR_INVALID_ARG = 1, MRTH_ERR_IO = 2, MRTH_ERR_GENERATOR = 3 };

typedef struct mrth_scene mrth_scene;
typedef struct mrth_bvh mrth_bvh;

typedef struct mrth_camera {
    float position[3];
    float forward[3];
    float up[3];
    float fov_deg;      /* vertical field of view */
    float near_dist;
    float far_dist;
} mrth_camera;

typedef struct mrth_build_params {
    float sah_node_cost;      /* 1.0 */
    float sah_triangle_cost;  /* 1.0 */
    int32_t min_leaf_size;    /* 1   (Renderer.cc:54) */
    int32_t max_leaf_size;    /* 8   (Renderer.cc:54) */
    float split_alpha;        /* 1e-5 (BVH.hh BuildParams) */
    int32_t threads;          /* 0 = all cores; output is independent of it */
} mrth_build_params;

typedef struct mrth_bvh_stats {
    int64_t inner_nodes;
    int64_t leaf_nodes;
    int64_t tri_refs;
    int64_t max_depth;
    float sah_cost;
    double build_seconds;
} mrth_bvh_stats;

/* ---- scenes -------------------------------------------------------------- */
/* name: "mori" | "bunny" | "conference" | "sponza" | "hairball" (published
 * triangle counts; "hairball" with param > 0: that many tubes, unpadded), "sphere" (param = rings), "random" (param = triangles). */
int  mrth_scene_synthetic(const char* name, int64_t param, uint64_t seed, mrth_scene** out);
int  mrth_scene_load_obj(const char* path, mrth_scene** out);
int  mrth_scene_from_arrays(const float* vertices, int64_t numVertices, const int32_t* triangles,
                            int64_t numTriangles, mrth_scene** out);
void mrth_scene_destroy(mrth_scene* s);
int64_t mrth_scene_num_triangles(const mrth_scene* s);
int64_t mrth_scene_num_vertices(const mrth_scene* s);
int  mrth_scene_copy_arrays(const mrth_scene* s, float* vertices /* 3*nv or NULL */,
                            int32_t* triangles /* 3*nt or NULL */, float* normals /* 3*nt or NULL */);
int  mrth_scene_camera(const mrth_scene* s, mrth_camera* cam, float* aoRadius);
/* Per-triangle ABGR colour tables of Scene::Scene (reference Scene.cc:47-80): the
 * material colour and the shaded colour diffuse * (dot(n, normalize(1,2,3)) / 2 + 1/2),
 * both through the host Vec4f::toABGR (Math.cc:45-52). A triangle's material is its OBJ
 * submesh's .mtl entry (Kd rgb, d alpha; MeshWavefrontIO.cc:114-200) or the default
 * (diffuse 0.75 grey, Mesh.hh:92; synthetic scenes). Either output may be NULL; each
 * holds num_triangles uint32. */
int  mrth_scene_tri_colors(const mrth_scene* s, uint32_t* material, uint32_t* shaded);

/* ---- BVH (SBVH build -> Compact2 host buffers) ---------------------------- */
void mrth_default_build_params(mrth_build_params* p);

/* hashBuffer (Hash.cc:34-76), the framework hash the two functions below are built on. */
uint32_t mrth_fw_hash_buffer(const void* ptr, int64_t size);
/* Scene::hash (Scene.cc:93-101): the framework hash (Hash.cc:34-76) of the scene's five
 * buffers — triangle vertex indices, face normals, material and shaded colours, positions. */
uint32_t mrth_scene_hash(const mrth_scene* s);
/* The reference's bvhcache file name for this scene and build (Renderer.cc:178-186):
 * "%08x.dat" of hashBits(scene hash, Platform("GPU") hash, BuildParams hash, BVHLayout_Compact2),
 * written to out (>= 13 bytes; 16 are touched). p NULL = defaults (mrth_default_build_params). */
int  mrth_bvh_cache_name(const mrth_scene* s, const mrth_build_params* p, char out[16]);
int  mrth_bvh_build(const mrth_scene* s, const mrth_build_params* p /* NULL = defaults */, mrth_bvh** out);
int  mrth_bvh_load(const char* datPath, mrth_bvh** out);
int  mrth_bvh_save(const mrth_bvh* b, const char* datPath);
int  mrth_bvh_from_buffers(const void* nodes, int64_t nodeBytes, const void* woop, int64_t woopBytes,
                           const int32_t* triIndex, int64_t triIndexBytes, mrth_bvh** out);
void mrth_bvh_destroy(mrth_bvh* b);
int  mrth_bvh_buffers(const mrth_bvh* b, const void** nodes, int64_t* nodeBytes, const void** woop,
                      int64_t* woopBytes, const int32_t** triIndex, int64_t* triIndexBytes);
int  mrth_bvh_get_stats(const mrth_bvh* b, mrth_bvh_stats* out);
/* Woop rows (Z,U,V; 12 floats) of one triangle, CudaBVH::woopifyTri. */
void mrth_woopify(const float v0[3], const float v1[3], const float v2[3], float out[12]);

/* ---- rays (Ray = 8 floats, RayResult = 4 x 32 bit) ------------------------ */
int  mrth_pixel_table(int32_t w, int32_t h, int32_t* indexToPixel /* w*h */);
int  mrth_primary_rays(const mrth_camera* cam, int32_t w, int32_t h, void* rays /* w*h Ray */,
                       int32_t* slotToId /* w*h or NULL */);
/* Primary rays sampled at (jx, jy) in [0, 1)^2 inside each pixel (centre = 0.5, 0.5). */
int  mrth_primary_rays_subpixel(const mrth_camera* cam, int32_t w, int32_t h, float jx, float jy, void* rays,
                                int32_t* slotToId);
/* CameraControls::decodeSignature (CameraControls.cc:374-419, 502-554): the 6-bit text
 * camera of the reference App's --camera argument (grtcmdline.txt). Fills cam (position,
 * forward, up, fov, near, far) and, if non-NULL, the signature's speed and keepAligned.
 * MRTH_ERR_INVALID_ARG for a malformed signature ("CameraControls: Invalid signature!"). */
int  mrth_camera_decode_signature(const char* sig, mrth_camera* cam, float* speed, int32_t* keepAligned);

/* invert(fitToView(-1, 2, (w, h)) * worldToClip), column-major (Renderer.cc:126-129): the
 * matrix mrt_raygen_primary (mrt.h) takes. */
int  mrth_camera_nscreen_to_world(const mrth_camera* cam, int32_t w, int32_t h, float out[16]);
int  mrth_ao_rays(const void* primaryRays, const void* primaryResults, int64_t numPrimary,
                  const mrth_scene* s, int32_t numSamples, float maxDist, uint32_t seed,
                  void* outRays /* numPrimary * numSamples Ray */);
int64_t mrth_count_hits(const void* results, int64_t n);

const char* mrth_last_error(void);

#ifdef __cplusplus
}
#endif

#endif /* MRT_HOST_H */
