/* gcs_store.h -- C ABI of the HDF5 trajectory store.
 *
 * Replaces the reference's simulation_store (src/simulation/common/simulation_store.{hpp,cpp}) and the h5 wrapper
 * under it with plain HDF5 primitives; the stage-level methods (save_positions, save_contacts, append_frame,
 * clear_frames, load_* designs) are composed from these by the host mirror (3d-genome-cycle_amd/gcs/store.py), with
 * the reference's dataset paths, types and filters:
 *   strings          variable-length, scalar or 1-D (".steps" is 1-D, chunked and extensible: rewritten on every
 *                    append_frame, simulation_store.cpp:177-189)
 *   positions        f32 (N, 3), deflate 6 (simulation_store.cpp:192-216)
 *   contacts         i32 (K, 3), deflate 4 + integer scale-offset, min bits 0 (simulation_store.cpp:253-267)
 *   particle_types   i32 enum (prepare.cpp:14-25)
 * Paths are absolute HDF5 paths; missing intermediate groups are created.  Writing a path that exists replaces it.
 * All functions return 0 on success, nonzero with gcs_store_last_error() set otherwise.  Not thread-safe.
 */
#ifndef GCS_STORE_H
#define GCS_STORE_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct gcs_store gcs_store;

#define GCS_H5_F32 1
#define GCS_H5_F64 2
#define GCS_H5_I32 3
#define GCS_H5_U32 4
#define GCS_H5_U64 5

const char* gcs_store_last_error(void);
/* create != 0: create (truncate) the file; otherwise open it read-write ("r+", simulation_store.cpp:63-66) */
int gcs_store_open(const char* path, int32_t create, gcs_store** out);
int gcs_store_close(gcs_store* s);
int gcs_store_flush(gcs_store* s);
int gcs_store_exists(gcs_store* s, const char* path, int32_t* exists);
int gcs_store_remove(gcs_store* s, const char* path);
int gcs_store_soft_link(gcs_store* s, const char* target, const char* link_path);

int gcs_store_write_string(gcs_store* s, const char* path, const char* text);
/* *len = bytes of the string (without NUL); copies min(len, cap - 1) bytes + NUL when cap > 0 */
int gcs_store_read_string(gcs_store* s, const char* path, char* buf, int64_t cap, int64_t* len);
int gcs_store_write_strings(gcs_store* s, const char* path, const char* const* items, int64_t count);
/* the strings NUL-separated into buf; *count items, *bytes total bytes incl. the NULs (call with cap 0 to size) */
int gcs_store_read_strings(gcs_store* s, const char* path, char* buf, int64_t cap, int64_t* count, int64_t* bytes);

/* rank 0 (scalar) to 2; deflate 0-9 (0 = none); scaleoffset_int != 0: integer scale-offset filter, min bits 0 */
int gcs_store_write_array(gcs_store* s, const char* path, int32_t dtype, int32_t rank, const int64_t* dims,
                          const void* data, int32_t deflate, int32_t scaleoffset_int);
/* rank 1 or 2, one chunk holding the whole array, deflate filter at level `deflate` (1-9), written from `zdata`: the
 * array (in the file type's byte order) already deflated by the caller into zlib format (compress2 at that level),
 * zbytes long.  The file is the one gcs_store_write_array(..., deflate, 0) writes; the caller can deflate frames on
 * several host threads while one thread owns the (not thread-safe) HDF5 library. */
int gcs_store_write_deflated(gcs_store* s, const char* path, int32_t dtype, int32_t rank, const int64_t* dims,
                             const void* zdata, int64_t zbytes, int32_t deflate);
/* i32 (rows, cols) with integer scale-offset + deflate (the contact tables' filters), chunks of chunk_rows rows
 * encoded on `threads` host threads (the library's filter encoding restated, byte-identical chunks) and written
 * with H5Dwrite_chunk; a chunk the restated encoder does not cover makes the library filter the array instead. */
int gcs_store_write_scaleoffset_i32(gcs_store* s, const char* path, const int32_t* data, int64_t rows, int32_t cols,
                                    int32_t deflate, int64_t chunk_rows, int32_t threads);
/* converts to dtype; dims[0..rank) out; cap_elems = capacity of buf in elements (0 to query) */
int gcs_store_read_array(gcs_store* s, const char* path, int32_t dtype, void* buf, int64_t cap_elems,
                         int32_t* rank, int64_t* dims);
/* i32 enum dataset with members names[k] = codes[k] */
int gcs_store_write_enum(gcs_store* s, const char* path, const int32_t* values, int64_t count,
                         const char* const* names, const int32_t* codes, int32_t ncodes);

#ifdef __cplusplus
}
#endif

#endif /* GCS_STORE_H */
