// gs_host.cpp -- host-side C++ of the hot path's inputs (no GPU work here):
//   * binary .ply loader + load-time activations   (src/Splats.cpp:174-344)
//   * .ply writer in save_ply's byte layout          (tests/plyFileGenerator.py:155-249)
//   * 3D covariance precompute                       (src/Splats.cpp:414-479)
//   * Camera uniforms, glm-free                      (src/Camera.cpp:19-65,181-212)
// All float expressions follow glm's operator order and are compiled with
// -ffp-contract=off, so they reproduce what the reference computes on the host.
#include "gs_internal.hpp"

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <string>
#include <vector>

namespace gs {

// ----------------------------------------------------------------- glm subset
// Column-major like glm: m[c*4 + r] / m[c][r].
struct Mat4 {
    float m[16];
    float &at(int c, int r) { return m[c * 4 + r]; }
    float at(int c, int r) const { return m[c * 4 + r]; }
    static Mat4 identity() {
        Mat4 o{};
        for (int i = 0; i < 4; ++i) o.at(i, i) = 1.f;
        return o;
    }
};

// glm operator*(mat4, mat4): Result[c] = A[0]*B[c][0] + A[1]*B[c][1] + A[2]*B[c][2] + A[3]*B[c][3]
static Mat4 mul(const Mat4 &a, const Mat4 &b) {
    Mat4 o{};
    for (int c = 0; c < 4; ++c)
        for (int r = 0; r < 4; ++r)
            o.at(c, r) = a.at(0, r) * b.at(c, 0) + a.at(1, r) * b.at(c, 1) + a.at(2, r) * b.at(c, 2) +
                         a.at(3, r) * b.at(c, 3);
    return o;
}

static float radians(float deg) { return deg * 0.01745329251994329576923690768489f; }

// glm::rotate(mat4 m, angle, axis) (gtc/matrix_transform.inl)
static Mat4 rotate(const Mat4 &m, float angle, float ax, float ay, float az) {
    const float c = std::cos(angle), s = std::sin(angle);
    const float len = std::sqrt(ax * ax + ay * ay + az * az);  // glm::normalize = v * inversesqrt(dot)
    const float inv = 1.f / len;
    const float axis[3] = {ax * inv, ay * inv, az * inv};
    const float temp[3] = {(1.f - c) * axis[0], (1.f - c) * axis[1], (1.f - c) * axis[2]};
    float R[3][3];
    R[0][0] = c + temp[0] * axis[0];
    R[0][1] = temp[0] * axis[1] + s * axis[2];
    R[0][2] = temp[0] * axis[2] - s * axis[1];
    R[1][0] = temp[1] * axis[0] - s * axis[2];
    R[1][1] = c + temp[1] * axis[1];
    R[1][2] = temp[1] * axis[2] + s * axis[0];
    R[2][0] = temp[2] * axis[0] + s * axis[1];
    R[2][1] = temp[2] * axis[1] - s * axis[0];
    R[2][2] = c + temp[2] * axis[2];
    Mat4 o{};
    for (int col = 0; col < 3; ++col)
        for (int r = 0; r < 4; ++r)
            o.at(col, r) = m.at(0, r) * R[col][0] + m.at(1, r) * R[col][1] + m.at(2, r) * R[col][2];
    for (int r = 0; r < 4; ++r) o.at(3, r) = m.at(3, r);
    return o;
}

// glm::translate(mat4 m, v): Result[3] = m[0]*v[0] + m[1]*v[1] + m[2]*v[2] + m[3]
static Mat4 translate(const Mat4 &m, float x, float y, float z) {
    Mat4 o = m;
    for (int r = 0; r < 4; ++r) o.at(3, r) = m.at(0, r) * x + m.at(1, r) * y + m.at(2, r) * z + m.at(3, r);
    return o;
}

// glm::perspective (RH, depth -1..1 -- glm's default clip space)
static Mat4 perspective(float fovy, float aspect, float zNear, float zFar) {
    const float tanHalfFovy = std::tan(fovy / 2.f);
    Mat4 o{};
    o.at(0, 0) = 1.f / (aspect * tanHalfFovy);
    o.at(1, 1) = 1.f / (tanHalfFovy);
    o.at(2, 2) = -(zFar + zNear) / (zFar - zNear);
    o.at(2, 3) = -1.f;
    o.at(3, 2) = -(2.f * zFar * zNear) / (zFar - zNear);
    return o;
}

// ------------------------------------------------------------------ loader
static bool read_line(std::FILE *f, std::string &line) {
    line.clear();
    int c;
    while ((c = std::fgetc(f)) != EOF && c != '\n') line.push_back(static_cast<char>(c));
    return !(c == EOF && line.empty());
}

int ply_count(const char *path, int *n) {
    std::FILE *f = std::fopen(path, "rb");
    if (!f) return set_error(nullptr, GS_ERR_IO, std::string("Error: failed to open file ") + path);
    std::string line;
    read_line(f, line);
    read_line(f, line);
    read_line(f, line);  // src/Splats.cpp:252-260: third line "element vertex N"
    std::fclose(f);
    char a[64], b[64];
    int v = -1;
    if (std::sscanf(line.c_str(), "%63s %63s %d", a, b, &v) != 3 || v < 0)
        return set_error(nullptr, GS_ERR_IO, std::string("Error: bad ply header in ") + path);
    *n = v;
    return GS_OK;
}

// the ply's vertex count and a FILE positioned at its body (src/Splats.cpp:252-267)
int ply_open_body(const char *path, int *n, std::FILE **out) {
    if (int rc = ply_count(path, n)) return rc;
    std::FILE *f = std::fopen(path, "rb");
    if (!f) return set_error(nullptr, GS_ERR_IO, std::string("Error: failed to open file ") + path);
    std::string line;
    for (int i = 0; i < 3; ++i) read_line(f, line);
    while (line != "end_header") {
        if (!read_line(f, line)) {
            std::fclose(f);
            return set_error(nullptr, GS_ERR_IO, "Error: no end_header in ply");
        }
    }
    *out = f;
    return GS_OK;
}

// One splat's activations (src/Splats.cpp:289-331); shared by the loader and gs_activate.
static inline void activate_one(const float *f_dc, float opac_logit, const float *log_scale,
                                const float *rot, float *colour4, float *opacity, float *scale3,
                                float *rot4) {
    const float SH_C0 = 0.28209479177387814f;
    if (colour4) {
        for (int c = 0; c < 3; ++c) colour4[c] = (0.5f + (SH_C0 * f_dc[c])) * 255.f;
        colour4[3] = 1.f;
    }
    if (opacity) *opacity = (1 / (1 + std::exp(-opac_logit)));
    if (scale3)
        for (int c = 0; c < 3; ++c) scale3[c] = std::exp(log_scale[c]);
    if (rot4) {
        const float length = std::sqrt(rot[0] * rot[0] + rot[1] * rot[1] + rot[2] * rot[2] + rot[3] * rot[3]);
        for (int c = 0; c < 4; ++c) rot4[c] = rot[c] / length;
    }
}

int ply_load(const char *path, int n, float *means4, float *colours4, float *opacity, float *scales3,
             float *rots4) {
    std::FILE *f = std::fopen(path, "rb");
    if (!f) return set_error(nullptr, GS_ERR_IO, std::string("Error: failed to open file ") + path);
    std::string line;
    for (int i = 0; i < 3; ++i) read_line(f, line);
    while (line != "end_header") {  // src/Splats.cpp:264-267
        if (!read_line(f, line)) {
            std::fclose(f);
            return set_error(nullptr, GS_ERR_IO, "Error: no end_header in ply");
        }
    }
    // body: 62 little-endian floats per splat, read in blocks
    const int kRec = 62;
    const int kBlock = 1 << 16;
    std::vector<float> buf(static_cast<size_t>(kBlock) * kRec);
    for (int base = 0; base < n; base += kBlock) {
        const int cnt = std::min(kBlock, n - base);
        if (std::fread(buf.data(), sizeof(float) * kRec, cnt, f) != static_cast<size_t>(cnt)) {
            std::fclose(f);
            return set_error(nullptr, GS_ERR_IO, "Error: failed to read all splats from file");
        }
        for (int j = 0; j < cnt; ++j) {
            const size_t i = static_cast<size_t>(base) + j;
            const float *rec = buf.data() + static_cast<size_t>(j) * kRec;
            if (means4) {
                means4[4 * i + 0] = rec[0];
                means4[4 * i + 1] = rec[1];
                means4[4 * i + 2] = rec[2];
                means4[4 * i + 3] = 1.f;
            }
            // rec[3..5] normal dropped, rec[9..53] f_rest read and discarded (Splats.cpp:286-302)
            activate_one(rec + 6, rec[54], rec + 55, rec + 58, colours4 ? colours4 + 4 * i : nullptr,
                         opacity ? opacity + i : nullptr, scales3 ? scales3 + 3 * i : nullptr,
                         rots4 ? rots4 + 4 * i : nullptr);
        }
    }
    const int extra = std::fgetc(f);  // :333-340 must be at EOF
    std::fclose(f);
    if (extra != EOF) return set_error(nullptr, GS_ERR_IO, "Error: failed to read all splats from file");
    return GS_OK;
}

int ply_load_sh(const char *path, int n, float *f_dc3, float *f_rest45) {
    int cnt_file = 0;
    std::FILE *f = nullptr;
    if (int rc = ply_open_body(path, &cnt_file, &f)) return rc;
    if (cnt_file != n) {
        std::fclose(f);
        return set_error(nullptr, GS_ERR_INVALID, "ply_load_sh: n differs from the file's vertex count");
    }
    const int kRec = 62, kBlock = 1 << 16;
    std::vector<float> buf(static_cast<size_t>(kBlock) * kRec);
    for (int base = 0; base < n; base += kBlock) {
        const int cnt = std::min(kBlock, n - base);
        if (std::fread(buf.data(), sizeof(float) * kRec, cnt, f) != static_cast<size_t>(cnt)) {
            std::fclose(f);
            return set_error(nullptr, GS_ERR_IO, "Error: failed to read all splats from file");
        }
        for (int j = 0; j < cnt; ++j) {
            const size_t i = static_cast<size_t>(base) + j;
            const float *rec = buf.data() + static_cast<size_t>(j) * kRec;
            if (f_dc3) std::memcpy(f_dc3 + 3 * i, rec + 6, 3 * sizeof(float));
            if (f_rest45) std::memcpy(f_rest45 + 45 * i, rec + 9, 45 * sizeof(float));
        }
    }
    std::fclose(f);
    return GS_OK;
}

int ply_write(const char *path, int n, const float *means3, const float *rots4, const float *scales3,
              const float *opacities, const float *colours3) {
    std::FILE *f = std::fopen(path, "wb");
    if (!f) return set_error(nullptr, GS_ERR_IO, std::string("Error: failed to open file ") + path);
    std::string hdr = "ply\nformat binary_little_endian 1.0\nelement vertex " + std::to_string(n) +
                      "\nproperty float x\nproperty float y\nproperty float z\nproperty float nx\n"
                      "property float ny\nproperty float nz\nproperty float f_dc_0\nproperty float f_dc_1\n"
                      "property float f_dc_2\n";
    for (int k = 0; k < 45; ++k) hdr += "property float f_rest_" + std::to_string(k) + "\n";
    hdr += "property float opacity\nproperty float scale_0\nproperty float scale_1\nproperty float scale_2\n"
           "property float rot_0\nproperty float rot_1\nproperty float rot_2\nproperty float rot_3\nend_header\n";
    std::fwrite(hdr.data(), 1, hdr.size(), f);
    std::vector<float> rec(62);
    for (int i = 0; i < n; ++i) {
        std::fill(rec.begin(), rec.end(), 0.f);
        for (int c = 0; c < 3; ++c) rec[c] = means3[3 * i + c];
        for (int c = 0; c < 3; ++c) rec[6 + c] = colours3[3 * i + c];
        const float o = opacities[i];
        rec[54] = std::log(o / (1 - o));  // np.log(o / (1 - o)) in float32
        for (int c = 0; c < 3; ++c) rec[55 + c] = std::log(scales3[3 * i + c]);
        for (int c = 0; c < 4; ++c) rec[58 + c] = rots4[4 * i + c];
        std::fwrite(rec.data(), sizeof(float), 62, f);
    }
    std::fclose(f);
    return GS_OK;
}

int activate(int n, const float *f_dc3, const float *opacity_logit, const float *log_scale3,
             const float *rot_raw4, float *colours4, float *opacity, float *scales3, float *rots4) {
    for (int i = 0; i < n; ++i)
        activate_one(f_dc3 + 3 * (size_t)i, opacity_logit[i], log_scale3 + 3 * (size_t)i,
                     rot_raw4 + 4 * (size_t)i, colours4 ? colours4 + 4 * (size_t)i : nullptr,
                     opacity ? opacity + i : nullptr, scales3 ? scales3 + 3 * (size_t)i : nullptr,
                     rots4 ? rots4 + 4 * (size_t)i : nullptr);
    return GS_OK;
}

// -------------------------------------------------------------- covariance
// src/Splats.cpp:440-479: T = S * R (glm mat3 product), Sigma = transpose(T) * T
int covariance3d(int n, const float *scales3, const float *rots4, float *cov6) {
    for (int i = 0; i < n; ++i) {
        const float S[3][3] = {{scales3[3 * i + 0], 0, 0}, {0, scales3[3 * i + 1], 0}, {0, 0, scales3[3 * i + 2]}};
        const float r = rots4[4 * i + 0], x = rots4[4 * i + 1], y = rots4[4 * i + 2], z = rots4[4 * i + 3];
        const float R[3][3] = {{1.f - 2.f * (y * y + z * z), 2.f * (x * y - r * z), 2.f * (x * z + r * y)},
                               {2.f * (x * y + r * z), 1.f - 2.f * (x * x + z * z), 2.f * (y * z - r * x)},
                               {2.f * (x * z - r * y), 2.f * (y * z + r * x), 1.f - 2.f * (x * x + y * y)}};
        float M[3][3], Mt[3][3], Sig[3][3];
        for (int c = 0; c < 3; ++c)
            for (int rr = 0; rr < 3; ++rr) M[c][rr] = S[0][rr] * R[c][0] + S[1][rr] * R[c][1] + S[2][rr] * R[c][2];
        for (int c = 0; c < 3; ++c)
            for (int rr = 0; rr < 3; ++rr) Mt[c][rr] = M[rr][c];
        for (int c = 0; c < 3; ++c)
            for (int rr = 0; rr < 3; ++rr)
                Sig[c][rr] = Mt[0][rr] * M[c][0] + Mt[1][rr] * M[c][1] + Mt[2][rr] * M[c][2];
        float *o = cov6 + 6 * (size_t)i;
        o[0] = Sig[0][0]; o[1] = Sig[0][1]; o[2] = Sig[0][2];
        o[3] = Sig[1][1]; o[4] = Sig[1][2]; o[5] = Sig[2][2];
    }
    return GS_OK;
}

// ------------------------------------------------------------------ camera
int camera_update(const gs_camera *cam, float view16[16], float proj16[16], float *focal_x, float *focal_y,
                  float *tan_fovx_getter, float *tan_fovy_getter) {
    // Camera::update (src/Camera.cpp:57-65)
    const Mat4 I = Mat4::identity();
    const Mat4 Rx = rotate(I, radians(cam->rotation[0]), 1.f, 0.f, 0.f);
    const Mat4 Ry = rotate(I, radians(cam->rotation[1]), 0.f, 1.f, 0.f);
    const Mat4 Rz = rotate(I, radians(cam->rotation[2]), 0.f, 0.f, 1.f);
    const Mat4 R3 = mul(mul(Rx, Ry), Rz);
    Mat4 rot = Mat4::identity();  // glm::mat4(glm::mat3(...)): upper-left 3x3, [3][3] = 1
    for (int c = 0; c < 3; ++c)
        for (int r = 0; r < 3; ++r) rot.at(c, r) = R3.at(c, r);
    const Mat4 T = translate(I, cam->position[0], cam->position[1], cam->position[2]);
    const Mat4 view = mul(rot, T);
    // Camera::setWidthHeight / constructor (src/Camera.cpp:19-30,49-55)
    const float aspect = (float)cam->width / (float)cam->height;
    const Mat4 proj = perspective(radians(cam->fovy), aspect, cam->near_plane, cam->far_plane);
    if (view16) std::memcpy(view16, view.m, sizeof(view.m));
    if (proj16) std::memcpy(proj16, proj.m, sizeof(proj.m));
    // getFocalX/Y (src/Camera.cpp:181-197): both divide by tan(fovy/2) (Q3)
    const float fovy_rad = radians(cam->fovy);
    if (focal_x) *focal_x = (float)cam->width / (2.0f * tanf(fovy_rad / 2.0f));
    if (focal_y) *focal_y = (float)cam->height / (2.0f * tanf(fovy_rad / 2.0f));
    // getTanFovx/y (src/Camera.cpp:199-212): fovy in DEGREES fed to tan (Q1);
    // `tan(fovy / 2.f)` resolves to ::tan(double) in Camera.cpp, tanf elsewhere.
    const float fovx = atanf((float)(::tan((double)(cam->fovy / 2.f)) * (double)aspect));
    if (tan_fovx_getter) *tan_fovx_getter = tanf(fovx);
    if (tan_fovy_getter) *tan_fovy_getter = tanf(cam->fovy / 2.0f);
    return GS_OK;
}

int camera_uniforms(const gs_camera *cam, gs_uniforms *u) {
    float proj[16], tx, ty;
    camera_update(cam, u->view, proj, &u->focal_x, &u->focal_y, &tx, &ty);
    Mat4 P, V;
    std::memcpy(P.m, proj, sizeof(proj));
    std::memcpy(V.m, u->view, sizeof(V.m));
    const Mat4 VP = mul(P, V);  // main.cpp:64 getProjectionMatrix() * getViewMatrix()
    std::memcpy(u->vp, VP.m, sizeof(VP.m));
    u->width = cam->width;
    u->height = cam->height;
    u->tan_fov_x = ty;  // main.cpp:63: camera.getTanFovy() passed as tan_fov_x (Q2)
    u->tan_fov_y = tx;  //              camera.getTanFovx() passed as tan_fov_y
    return GS_OK;
}

// ------------------------------------------------------------------ image dump
// saveImage (src/Splats.cpp:516-540) writes an RGBA PNG whose row h is pixel row y = h of
// the render, i.e. row 0 = the GL bottom row; flip_y = 1 writes the screen orientation
// instead.  Self-contained writer: zlib stream of stored (uncompressed) deflate blocks.
namespace {
uint32_t crc32_png(const uint8_t *p, size_t n, uint32_t c = 0xffffffffu) {
    static uint32_t table[256];
    static bool init = false;
    if (!init) {
        for (uint32_t i = 0; i < 256; ++i) {
            uint32_t v = i;
            for (int k = 0; k < 8; ++k) v = (v & 1) ? 0xedb88320u ^ (v >> 1) : v >> 1;
            table[i] = v;
        }
        init = true;
    }
    for (size_t i = 0; i < n; ++i) c = table[(c ^ p[i]) & 0xff] ^ (c >> 8);
    return c;
}
void put_be32(std::vector<uint8_t> &v, uint32_t x) {
    for (int s = 24; s >= 0; s -= 8) v.push_back((uint8_t)(x >> s));
}
void png_chunk(std::vector<uint8_t> &out, const char *type, const std::vector<uint8_t> &data) {
    put_be32(out, (uint32_t)data.size());
    const size_t at = out.size();
    out.insert(out.end(), type, type + 4);
    out.insert(out.end(), data.begin(), data.end());
    put_be32(out, crc32_png(out.data() + at, data.size() + 4) ^ 0xffffffffu);
}
}  // namespace

int save_png(const char *path, int width, int height, const uint8_t *rgba8, int flip_y) {
    if (!path || !rgba8 || width <= 0 || height <= 0) return set_error(nullptr, GS_ERR_INVALID, "save_png: bad argument");
    const size_t row = (size_t)width * 4;
    std::vector<uint8_t> raw;  // filter byte 0 + row
    raw.reserve((row + 1) * height);
    for (int h = 0; h < height; ++h) {
        const int y = flip_y ? height - 1 - h : h;
        raw.push_back(0);
        raw.insert(raw.end(), rgba8 + (size_t)y * row, rgba8 + (size_t)(y + 1) * row);
    }
    std::vector<uint8_t> z = {0x78, 0x01};  // zlib header, no compression
    uint32_t a = 1, b = 0;                   // adler32
    for (uint8_t c : raw) {
        a = (a + c) % 65521u;
        b = (b + a) % 65521u;
    }
    for (size_t off = 0; off < raw.size() || off == 0;) {
        const size_t len = std::min<size_t>(65535, raw.size() - off);
        const bool last = off + len >= raw.size();
        z.push_back(last ? 1 : 0);
        z.push_back((uint8_t)(len & 0xff));
        z.push_back((uint8_t)(len >> 8));
        z.push_back((uint8_t)(~len & 0xff));
        z.push_back((uint8_t)((~len >> 8) & 0xff));
        z.insert(z.end(), raw.begin() + off, raw.begin() + off + len);
        off += len;
        if (last) break;
    }
    put_be32(z, (b << 16) | a);
    std::vector<uint8_t> out = {0x89, 'P', 'N', 'G', '\r', '\n', 0x1a, '\n'};
    std::vector<uint8_t> ihdr;
    put_be32(ihdr, (uint32_t)width);
    put_be32(ihdr, (uint32_t)height);
    ihdr.insert(ihdr.end(), {8, 6, 0, 0, 0});  // 8-bit RGBA, deflate, adaptive filter, no interlace
    png_chunk(out, "IHDR", ihdr);
    png_chunk(out, "IDAT", z);
    png_chunk(out, "IEND", {});
    FILE *f = std::fopen(path, "wb");
    if (!f) return set_error(nullptr, GS_ERR_IO, std::string("save_png: cannot open ") + path);
    const bool ok = std::fwrite(out.data(), 1, out.size(), f) == out.size();
    std::fclose(f);
    return ok ? GS_OK : set_error(nullptr, GS_ERR_IO, std::string("save_png: write failed: ") + path);
}

}  // namespace gs
