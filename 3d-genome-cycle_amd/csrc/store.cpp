// store.cpp -- HDF5 trajectory store primitives (include/gcs_store.h) over the HDF5 C library.
//
// Host-only: the store is off the step loop.  The reference's simulation_store sits on the h5
// header library (an absent submodule); this file keeps its on-disk contract (Appendix A of SURVEY.md), which the
// Python tools (dumpgsd.py, cool.py) read: vlen strings, f32 positions with deflate 6, i32 contacts with deflate 4 +
// integer scale-offset, an i32 enum for particle_types, soft links between stage metadata groups.
#include <hdf5.h>
#include <zlib.h>

#include <algorithm>
#include <cstring>
#include <string>
#include <thread>
#include <vector>

#include "../../include/gcs_store.h"

namespace {

thread_local std::string g_err;

int fail(const std::string& m)
{
    g_err = m;
    return 1;
}

struct Silence {  // no HDF5 error stack printing: errors come back as status codes + gcs_store_last_error
    H5E_auto2_t fn = nullptr;
    void* data = nullptr;
    Silence()
    {
        H5Eget_auto2(H5E_DEFAULT, &fn, &data);
        H5Eset_auto2(H5E_DEFAULT, nullptr, nullptr);
    }
    ~Silence() { H5Eset_auto2(H5E_DEFAULT, fn, data); }
};

hid_t mem_type(int dtype)
{
    switch (dtype) {
    case GCS_H5_F32: return H5T_NATIVE_FLOAT;
    case GCS_H5_F64: return H5T_NATIVE_DOUBLE;
    case GCS_H5_I32: return H5T_NATIVE_INT32;
    case GCS_H5_U32: return H5T_NATIVE_UINT32;
    case GCS_H5_U64: return H5T_NATIVE_UINT64;
    default: return -1;
    }
}

hid_t file_type(int dtype)
{
    switch (dtype) {
    case GCS_H5_F32: return H5T_IEEE_F32LE;
    case GCS_H5_F64: return H5T_IEEE_F64LE;
    case GCS_H5_I32: return H5T_STD_I32LE;
    case GCS_H5_U32: return H5T_STD_U32LE;
    case GCS_H5_U64: return H5T_STD_U64LE;
    default: return -1;
    }
}


hid_t vlen_str()
{
    hid_t t = H5Tcopy(H5T_C_S1);
    H5Tset_size(t, H5T_VARIABLE);
    H5Tset_cset(t, H5T_CSET_UTF8);
    return t;
}

// every missing parent group is created by the link-creation property
hid_t lcpl_parents()
{
    hid_t p = H5Pcreate(H5P_LINK_CREATE);
    H5Pset_create_intermediate_group(p, 1);
    return p;
}

bool path_exists(hid_t file, const std::string& path)
{
    // H5Lexists needs every intermediate link to exist: walk the components
    size_t pos = 1;
    while (true) {
        size_t next = path.find('/', pos);
        std::string part = path.substr(0, next);
        if (H5Lexists(file, part.c_str(), H5P_DEFAULT) <= 0) return false;
        if (next == std::string::npos) return true;
        pos = next + 1;
    }
}

int replace(hid_t file, const std::string& path)
{
    if (path_exists(file, path) && H5Ldelete(file, path.c_str(), H5P_DEFAULT) < 0)
        return fail("cannot replace " + path);
    return 0;
}

}  // namespace

struct gcs_store {
    hid_t file = -1;
};

extern "C" {

const char* gcs_store_last_error(void) { return g_err.c_str(); }

int gcs_store_open(const char* path, int32_t create, gcs_store** out)
{
    if (!path || !out) return fail("null argument");
    Silence q;
    *out = nullptr;
    hid_t f = create ? H5Fcreate(path, H5F_ACC_TRUNC, H5P_DEFAULT, H5P_DEFAULT)
                     : H5Fopen(path, H5F_ACC_RDWR, H5P_DEFAULT);
    if (f < 0) return fail(std::string("cannot open HDF5 file ") + path);
    auto* s = new gcs_store();
    s->file = f;
    *out = s;
    return 0;
}

int gcs_store_close(gcs_store* s)
{
    if (!s) return 0;
    int rc = 0;
    if (s->file >= 0 && H5Fclose(s->file) < 0) rc = fail("H5Fclose failed");
    delete s;
    return rc;
}

int gcs_store_flush(gcs_store* s)
{
    if (!s) return fail("null argument");
    return H5Fflush(s->file, H5F_SCOPE_GLOBAL) < 0 ? fail("H5Fflush failed") : 0;
}

int gcs_store_exists(gcs_store* s, const char* path, int32_t* exists)
{
    if (!s || !path || !exists) return fail("null argument");
    Silence q;
    *exists = path_exists(s->file, path) ? 1 : 0;
    // a dangling soft link is not a dataset
    if (*exists && H5Oexists_by_name(s->file, path, H5P_DEFAULT) <= 0) *exists = 0;
    return 0;
}

int gcs_store_remove(gcs_store* s, const char* path)
{
    if (!s || !path) return fail("null argument");
    Silence q;
    return replace(s->file, path);
}

int gcs_store_soft_link(gcs_store* s, const char* target, const char* link_path)
{
    if (!s || !target || !link_path) return fail("null argument");
    Silence q;
    if (replace(s->file, link_path)) return 1;
    hid_t lp = lcpl_parents();
    herr_t e = H5Lcreate_soft(target, s->file, link_path, lp, H5P_DEFAULT);
    H5Pclose(lp);
    return e < 0 ? fail(std::string("cannot link ") + link_path) : 0;
}

int gcs_store_write_string(gcs_store* s, const char* path, const char* text)
{
    if (!s || !path || !text) return fail("null argument");
    Silence q;
    if (replace(s->file, path)) return 1;
    hid_t t = vlen_str(), sp = H5Screate(H5S_SCALAR), lp = lcpl_parents();
    hid_t d = H5Dcreate2(s->file, path, t, sp, lp, H5P_DEFAULT, H5P_DEFAULT);
    int rc = 0;
    if (d < 0 || H5Dwrite(d, t, H5S_ALL, H5S_ALL, H5P_DEFAULT, &text) < 0) rc = fail(std::string("cannot write ") + path);
    if (d >= 0) H5Dclose(d);
    H5Pclose(lp);
    H5Sclose(sp);
    H5Tclose(t);
    return rc;
}

int gcs_store_read_string(gcs_store* s, const char* path, char* buf, int64_t cap, int64_t* len)
{
    if (!s || !path || !len || (cap > 0 && !buf)) return fail("null argument");
    Silence q;
    hid_t d = H5Dopen2(s->file, path, H5P_DEFAULT);
    if (d < 0) return fail(std::string("no dataset ") + path);
    hid_t ft = H5Dget_type(d);
    int rc = 0;
    std::string out;
    if (H5Tis_variable_str(ft) > 0) {
        hid_t t = vlen_str();
        char* p = nullptr;
        if (H5Dread(d, t, H5S_ALL, H5S_ALL, H5P_DEFAULT, &p) < 0)
            rc = fail(std::string("cannot read ") + path);
        else if (p) {
            out = p;
            hid_t sp = H5Dget_space(d);
            H5Dvlen_reclaim(t, sp, H5P_DEFAULT, &p);
            H5Sclose(sp);
        }
        H5Tclose(t);
    } else {  // fixed-length string
        const size_t n = H5Tget_size(ft);
        std::vector<char> tmp(n + 1, 0);
        hid_t t = H5Tcopy(H5T_C_S1);
        H5Tset_size(t, n);
        if (H5Dread(d, t, H5S_ALL, H5S_ALL, H5P_DEFAULT, tmp.data()) < 0) rc = fail(std::string("cannot read ") + path);
        out.assign(tmp.data());
        H5Tclose(t);
    }
    H5Tclose(ft);
    H5Dclose(d);
    if (rc) return rc;
    *len = (int64_t)out.size();
    if (cap > 0) {
        const size_t c = std::min<size_t>(out.size(), (size_t)cap - 1);
        std::memcpy(buf, out.data(), c);
        buf[c] = 0;
    }
    return 0;
}

int gcs_store_write_strings(gcs_store* s, const char* path, const char* const* items, int64_t count)
{
    if (!s || !path || (count > 0 && !items)) return fail("null argument");
    Silence q;
    if (replace(s->file, path)) return 1;
    hsize_t dims[1] = {(hsize_t)count}, maxd[1] = {H5S_UNLIMITED}, chunk[1] = {64};
    hid_t t = vlen_str(), sp = H5Screate_simple(1, dims, maxd), lp = lcpl_parents(), cp = H5Pcreate(H5P_DATASET_CREATE);
    H5Pset_chunk(cp, 1, chunk);
    hid_t d = H5Dcreate2(s->file, path, t, sp, lp, cp, H5P_DEFAULT);
    int rc = 0;
    if (d < 0 || (count > 0 && H5Dwrite(d, t, H5S_ALL, H5S_ALL, H5P_DEFAULT, items) < 0))
        rc = fail(std::string("cannot write ") + path);
    if (d >= 0) H5Dclose(d);
    H5Pclose(cp);
    H5Pclose(lp);
    H5Sclose(sp);
    H5Tclose(t);
    return rc;
}

int gcs_store_read_strings(gcs_store* s, const char* path, char* buf, int64_t cap, int64_t* count, int64_t* bytes)
{
    if (!s || !path || !count || !bytes || (cap > 0 && !buf)) return fail("null argument");
    Silence q;
    hid_t d = H5Dopen2(s->file, path, H5P_DEFAULT);
    if (d < 0) return fail(std::string("no dataset ") + path);
    hid_t sp = H5Dget_space(d);
    const hssize_t n = H5Sget_simple_extent_npoints(sp);
    hid_t t = vlen_str();
    std::vector<char*> p((size_t)std::max<hssize_t>(n, 1), nullptr);
    int rc = 0;
    if (n > 0 && H5Dread(d, t, H5S_ALL, H5S_ALL, H5P_DEFAULT, p.data()) < 0) rc = fail(std::string("cannot read ") + path);
    std::string all;
    if (!rc)
        for (hssize_t k = 0; k < n; ++k) {
            all += p[k] ? p[k] : "";
            all.push_back('\0');
        }
    if (n > 0 && !rc) H5Dvlen_reclaim(t, sp, H5P_DEFAULT, p.data());
    H5Tclose(t);
    H5Sclose(sp);
    H5Dclose(d);
    if (rc) return rc;
    *count = n;
    *bytes = (int64_t)all.size();
    if (cap > 0) std::memcpy(buf, all.data(), std::min<size_t>(all.size(), (size_t)cap));
    return 0;
}

int gcs_store_write_array(gcs_store* s, const char* path, int32_t dtype, int32_t rank, const int64_t* dims,
                          const void* data, int32_t deflate, int32_t scaleoffset_int)
{
    if (!s || !path || (rank > 0 && !dims)) return fail("null argument");
    if (rank < 0 || rank > 2) return fail("rank must be 0, 1 or 2");
    const hid_t mt = mem_type(dtype), ft = file_type(dtype);
    if (mt < 0) return fail("unknown dtype");
    Silence q;
    if (replace(s->file, path)) return 1;
    hsize_t hd[2] = {0, 0};
    hsize_t total = 1;
    for (int k = 0; k < rank; ++k) {
        hd[k] = (hsize_t)dims[k];
        total *= hd[k];
    }
    if (total > 0 && !data) return fail("null data");
    hid_t sp = rank == 0 ? H5Screate(H5S_SCALAR) : H5Screate_simple(rank, hd, nullptr);
    hid_t cp = H5Pcreate(H5P_DATASET_CREATE);
    const bool filtered = rank > 0 && total > 0 && (deflate > 0 || scaleoffset_int);
    if (filtered) {
        H5Pset_chunk(cp, rank, hd);  // one chunk: the arrays are written and read whole
        if (scaleoffset_int) H5Pset_scaleoffset(cp, H5Z_SO_INT, H5Z_SO_INT_MINBITS_DEFAULT);
        if (deflate > 0) H5Pset_deflate(cp, (unsigned)deflate);
    }
    hid_t lp = lcpl_parents();
    hid_t d = H5Dcreate2(s->file, path, ft, sp, lp, cp, H5P_DEFAULT);
    int rc = 0;
    if (d < 0 || (total > 0 && H5Dwrite(d, mt, H5S_ALL, H5S_ALL, H5P_DEFAULT, data) < 0))
        rc = fail(std::string("cannot write ") + path);
    if (d >= 0) H5Dclose(d);
    H5Pclose(lp);
    H5Pclose(cp);
    H5Sclose(sp);
    return rc;
}

int gcs_store_write_deflated(gcs_store* s, const char* path, int32_t dtype, int32_t rank, const int64_t* dims,
                             const void* zdata, int64_t zbytes, int32_t deflate)
{
    if (!s || !path || !dims || !zdata) return fail("null argument");
    if (rank < 1 || rank > 2) return fail("rank must be 1 or 2");
    if (deflate < 1 || deflate > 9) return fail("deflate level must be in [1, 9]");
    if (zbytes <= 0) return fail("empty compressed chunk");
    const hid_t ft = file_type(dtype);
    if (ft < 0) return fail("unknown dtype");
    Silence q;
    if (replace(s->file, path)) return 1;
    hsize_t hd[2] = {0, 0};
    for (int k = 0; k < rank; ++k) {
        hd[k] = (hsize_t)dims[k];
        if (hd[k] == 0) return fail("empty array");
    }
    hid_t sp = H5Screate_simple(rank, hd, nullptr);
    hid_t cp = H5Pcreate(H5P_DATASET_CREATE);
    H5Pset_chunk(cp, rank, hd);  // one chunk, as gcs_store_write_array lays a filtered array out
    H5Pset_deflate(cp, (unsigned)deflate);
    hid_t lp = lcpl_parents();
    hid_t d = H5Dcreate2(s->file, path, ft, sp, lp, cp, H5P_DEFAULT);
    const hsize_t off[2] = {0, 0};
    int rc = 0;
    // filter mask 0: every filter of the pipeline (deflate) was applied to the chunk
    if (d < 0 || H5Dwrite_chunk(d, H5P_DEFAULT, 0u, off, (size_t)zbytes, zdata) < 0)
        rc = fail(std::string("cannot write ") + path);
    if (d >= 0) H5Dclose(d);
    H5Pclose(lp);
    H5Pclose(cp);
    H5Sclose(sp);
    return rc;
}

namespace {
// HDF5's integer scale-offset filter (H5Z_SO_INT, minimum bits computed by the library) on one chunk of i32 values,
// as the library encodes it when the dataset's fill value (0, the default) is defined: the fill value is kept out of
// the min / max and coded as the all-ones code, every other value as (v - min) in minbits = ceil(log2(range + 2))
// bits, packed most significant bit first; a 21-byte header {minbits u32 LE, 8, min as i64 LE, 8 zero bytes}; the
// packed buffer is n * minbits / 8 + 1 bytes.  Checked byte for byte against the library's chunks
// (tests/test_store.py).  Empty result: a chunk the encoder does not cover (only fill values, or 32 bits needed).
std::vector<unsigned char> scaleoffset_i32(const int32_t* v, size_t n)
{
    bool any = false;
    long long mn = 0, mx = 0;
    for (size_t k = 0; k < n; ++k)
        if (v[k] != 0) {
            if (!any || v[k] < mn) mn = v[k];
            if (!any || v[k] > mx) mx = v[k];
            any = true;
        }
    if (!any) return {};
    const unsigned long long range = (unsigned long long)(mx - mn);
    int minbits = 0;
    while (minbits < 32 && (1ull << minbits) < range + 2) ++minbits;
    if (minbits >= 32) return {};
    std::vector<unsigned char> out(21 + n * (size_t)minbits / 8 + 1, 0);
    const unsigned mb = (unsigned)minbits;
    for (int b = 0; b < 4; ++b) out[b] = (unsigned char)(mb >> (8 * b));
    out[4] = 8;
    for (int b = 0; b < 8; ++b) out[5 + b] = (unsigned char)((unsigned long long)mn >> (8 * b));
    const unsigned long long fillcode = (1ull << minbits) - 1ull;
    unsigned char* d = out.data() + 21;
    unsigned long long acc = 0;  // pending bits, the oldest highest (MSB-first stream)
    int nb = 0;
    for (size_t k = 0; k < n; ++k) {
        const unsigned long long c = v[k] == 0 ? fillcode : (unsigned long long)((long long)v[k] - mn);
        acc = (acc << minbits) | c;  // nb < 8 before: at most 39 bits held
        nb += minbits;
        while (nb >= 8) {
            nb -= 8;
            *d++ = (unsigned char)(acc >> nb);
        }
        acc &= (1ull << nb) - 1ull;
    }
    if (nb > 0) *d = (unsigned char)(acc << (8 - nb));
    return out;
}
}  // namespace

int gcs_store_write_scaleoffset_i32(gcs_store* s, const char* path, const int32_t* data, int64_t rows, int32_t cols,
                                    int32_t deflate, int64_t chunk_rows, int32_t threads)
{
    if (!s || !path || !data) return fail("null argument");
    if (rows <= 0 || cols <= 0 || chunk_rows <= 0) return fail("rows, columns and chunk rows must be positive");
    if (deflate < 1 || deflate > 9) return fail("deflate level must be in [1, 9]");
    const int64_t cr = std::min(rows, chunk_rows);
    const int64_t nchunk = (rows + cr - 1) / cr;
    // encode every chunk (edge chunks padded with the fill value, as the library stores them) on `threads` threads
    std::vector<std::vector<unsigned char>> z((size_t)nchunk);
    std::vector<int> bad((size_t)nchunk, 0);
    auto work = [&](int64_t c0, int64_t step) {
        std::vector<int32_t> buf((size_t)(cr * cols));
        for (int64_t c = c0; c < nchunk; c += step) {
            const int64_t r0 = c * cr, nr = std::min(cr, rows - r0);
            std::fill(buf.begin(), buf.end(), 0);
            std::memcpy(buf.data(), data + r0 * cols, (size_t)(nr * cols) * sizeof(int32_t));
            const std::vector<unsigned char> so = scaleoffset_i32(buf.data(), buf.size());
            if (so.empty()) {
                bad[(size_t)c] = 1;
                continue;
            }
            // the library's deflate filter: compress2 into so.size() * 1.001 + 12 bytes, or the filter fails
            uLongf cap = (uLongf)((double)so.size() * 1.001 + 12);
            std::vector<unsigned char> out(cap);
            if (compress2(out.data(), &cap, so.data(), (uLong)so.size(), deflate) != Z_OK) {
                bad[(size_t)c] = 1;
                continue;
            }
            out.resize(cap);
            z[(size_t)c] = std::move(out);
        }
    };
    const int64_t nt = std::max<int64_t>(1, std::min<int64_t>({(int64_t)std::max(threads, 1), nchunk, 64}));
    std::vector<std::thread> pool;
    for (int64_t t = 1; t < nt; ++t) pool.emplace_back(work, t, nt);
    work(0, nt);
    for (auto& t : pool) t.join();
    const bool direct = std::find(bad.begin(), bad.end(), 1) == bad.end();

    Silence q;
    if (replace(s->file, path)) return 1;
    hsize_t hd[2] = {(hsize_t)rows, (hsize_t)cols}, ch[2] = {(hsize_t)cr, (hsize_t)cols};
    hid_t sp = H5Screate_simple(2, hd, nullptr);
    hid_t cp = H5Pcreate(H5P_DATASET_CREATE);
    H5Pset_chunk(cp, 2, ch);
    H5Pset_scaleoffset(cp, H5Z_SO_INT, H5Z_SO_INT_MINBITS_DEFAULT);
    H5Pset_deflate(cp, (unsigned)deflate);
    hid_t lp = lcpl_parents();
    hid_t d = H5Dcreate2(s->file, path, H5T_STD_I32LE, sp, lp, cp, H5P_DEFAULT);
    int rc = d < 0 ? fail(std::string("cannot create ") + path) : 0;
    if (!rc && !direct) {  // some chunk the encoder does not cover: the library filters the whole array
        if (H5Dwrite(d, H5T_NATIVE_INT32, H5S_ALL, H5S_ALL, H5P_DEFAULT, data) < 0)
            rc = fail(std::string("cannot write ") + path);
    }
    for (int64_t c = 0; !rc && direct && c < nchunk; ++c) {
        const hsize_t off[2] = {(hsize_t)(c * cr), 0};
        if (H5Dwrite_chunk(d, H5P_DEFAULT, 0u, off, z[(size_t)c].size(), z[(size_t)c].data()) < 0)
            rc = fail(std::string("cannot write a chunk of ") + path);
    }
    if (d >= 0) H5Dclose(d);
    H5Pclose(lp);
    H5Pclose(cp);
    H5Sclose(sp);
    return rc;
}

int gcs_store_read_array(gcs_store* s, const char* path, int32_t dtype, void* buf, int64_t cap_elems, int32_t* rank,
                         int64_t* dims)
{
    if (!s || !path || !rank || !dims || (cap_elems > 0 && !buf)) return fail("null argument");
    const hid_t mt = mem_type(dtype);
    if (mt < 0) return fail("unknown dtype");
    Silence q;
    hid_t d = H5Dopen2(s->file, path, H5P_DEFAULT);
    if (d < 0) return fail(std::string("no dataset ") + path);
    hid_t sp = H5Dget_space(d);
    const int r = H5Sget_simple_extent_ndims(sp);
    hsize_t hd[8] = {0};
    H5Sget_simple_extent_dims(sp, hd, nullptr);
    int64_t total = 1;
    for (int k = 0; k < r; ++k) total *= (int64_t)hd[k];
    *rank = r;
    for (int k = 0; k < r && k < 2; ++k) dims[k] = (int64_t)hd[k];
    int rc = 0;
    if (r > 2)
        rc = fail("rank > 2");
    else if (cap_elems > 0) {
        if (total > cap_elems)
            rc = fail("buffer too small");
        else if (total > 0 && H5Dread(d, mt, H5S_ALL, H5S_ALL, H5P_DEFAULT, buf) < 0)
            rc = fail(std::string("cannot read ") + path);
    }
    H5Sclose(sp);
    H5Dclose(d);
    return rc;
}

int gcs_store_write_enum(gcs_store* s, const char* path, const int32_t* values, int64_t count,
                         const char* const* names, const int32_t* codes, int32_t ncodes)
{
    if (!s || !path || (count > 0 && !values) || (ncodes > 0 && (!names || !codes))) return fail("null argument");
    Silence q;
    if (replace(s->file, path)) return 1;
    hid_t et = H5Tenum_create(H5T_STD_I32LE);
    for (int k = 0; k < ncodes; ++k) {
        const int32_t v = codes[k];
        H5Tenum_insert(et, names[k], &v);
    }
    hsize_t hd[1] = {(hsize_t)count};
    hid_t sp = H5Screate_simple(1, hd, nullptr), lp = lcpl_parents();
    hid_t d = H5Dcreate2(s->file, path, et, sp, lp, H5P_DEFAULT, H5P_DEFAULT);
    int rc = 0;
    // memory type: the same enum over native int32 (values are the codes)
    hid_t mt = H5Tenum_create(H5T_NATIVE_INT32);
    for (int k = 0; k < ncodes; ++k) {
        const int32_t v = codes[k];
        H5Tenum_insert(mt, names[k], &v);
    }
    if (d < 0 || (count > 0 && H5Dwrite(d, mt, H5S_ALL, H5S_ALL, H5P_DEFAULT, values) < 0))
        rc = fail(std::string("cannot write ") + path);
    if (d >= 0) H5Dclose(d);
    H5Tclose(mt);
    H5Pclose(lp);
    H5Sclose(sp);
    H5Tclose(et);
    return rc;
}

}  // extern "C"
