// gsplat_splats.hpp -- header-only C++ facade over include/gsplat.h that keeps the
// reference's C++ API for the hot path (thomas-chernaik/OpenGLGaussianSplattingRenderer):
//
//   include/Splats.h:29-124  class Splats   (constructor, gpuRender, sort, computeBins, draw,
//                                            display, public host vectors)
//   include/sort.h:15-23     GPURadixSort, PadBuffer, createAndLinkSortAndHistogramShaders
//
// GL object handles become device pointers / a context; glm::mat4 becomes gs::mat4 (the same
// column-major float[16] layout, indexed m[c][r] like glm).  Errors print the reference's
// messages to std::cerr and continue, as the reference does (src/sort.cpp:150-154,
// src/Splats.cpp:245-249); status codes are also returned for callers that check them.
#pragma once

#include <cstdint>
#include <cstring>
#include <iostream>
#include <memory>
#include <mutex>
#include <string>
#include <unordered_map>
#include <vector>

#include "gsplat.h"

namespace gs {

struct mat4 {
    float m[4][4];  // m[column][row], like glm::mat4
    const float *data() const { return &m[0][0]; }
};
struct vec3 {
    float x, y, z;
};
struct vec4 {
    float x, y, z, w;
};

inline int report(int rc, const gs_ctx *ctx = nullptr) {
    if (rc < 0) std::cerr << "Error: " << gs_last_error(ctx) << std::endl;
    return rc;
}

// One GPU: replaces the GL context + compiled programs.  Like a GL context it can be made
// current on the calling thread (the first one created is), so the reference's context-free
// calls -- GPURadixSort's 10-argument form -- find it.  A thread's current Context is held as
// (pointer, serial) and checked against a process-wide registry of live contexts, so a Context
// destroyed on another thread (or a new one at the same address) is never returned.
class Context {
  public:
    explicit Context(int device = 0) {
        report(gs_ctx_create(device, &ctx_));
        {
            std::lock_guard<std::mutex> g(registry_mutex());
            serial_ = ++serial_counter();
            registry()[this] = serial_;
        }
        if (!current()) makeCurrent();
    }
    ~Context() {
        {
            std::lock_guard<std::mutex> g(registry_mutex());
            registry().erase(this);
        }
        if (current_slot().ctx == this) current_slot() = Slot{};
        gs_ctx_destroy(ctx_);
    }
    Context(const Context &) = delete;
    Context &operator=(const Context &) = delete;
    gs_ctx *get() const { return ctx_; }
    void makeCurrent() { current_slot() = Slot{this, serial_}; }  // glfwMakeContextCurrent
    // the calling thread's current Context, or null (none made current, or it was destroyed)
    static Context *current() {
        const Slot s = current_slot();
        if (!s.ctx) return nullptr;
        std::lock_guard<std::mutex> g(registry_mutex());
        const auto it = registry().find(s.ctx);
        return (it != registry().end() && it->second == s.serial) ? s.ctx : nullptr;
    }
    void finish() const { report(gs_sync(ctx_), ctx_); }  // glFinish
    // frames in flight on the device: 2 (default; frame k+1's preprocess / emission / sort
    // overlap frame k's blend), 3 (one more in flight), or 1 (one frame at a time, as
    // gpuRender blocks)
    int setLanes(int lanes) const { return report(gs_ctx_set_lanes(ctx_, lanes), ctx_); }

  private:
    struct Slot {
        Context *ctx = nullptr;
        uint64_t serial = 0;
    };
    static Slot &current_slot() {
        static thread_local Slot cur;
        return cur;
    }
    static std::mutex &registry_mutex() {
        static std::mutex m;
        return m;
    }
    static std::unordered_map<const Context *, uint64_t> &registry() {
        static std::unordered_map<const Context *, uint64_t> r;
        return r;
    }
    static uint64_t &serial_counter() {
        static uint64_t c = 0;
        return c;
    }
    gs_ctx *ctx_ = nullptr;
    uint64_t serial_ = 0;
};

// src/sort.cpp:15-124 -- kernels are built ahead of time; nothing to compile.
inline void createAndLinkSortAndHistogramShaders(unsigned &histogramProgram, unsigned &sortProgram,
                                                 unsigned &sumProgram) {
    std::cout << "compiling sorting shaders" << std::endl;
    histogramProgram = 1;
    sortProgram = 2;
    sumProgram = 3;
    std::cout << "compiled and linked sorting shaders" << std::endl;
}

// src/sort.cpp:127-137
inline int PadBuffer(int size, int unitWidth) { return gs_pad_buffer(size, unitWidth); }

// src/sort.cpp:139-203.  orderBuffer (int32[size], device) is read as the initial order and
// receives the stable order of keysBuffer (float[size], device) by floatBitsToUint; the keys
// are not moved.  Program handles, intermediate / histogram buffers and the workgroup shape
// are accepted for signature parity (the HIP sort keeps its own scratch in the context).
inline int GPURadixSort(const Context &ctx, unsigned /*histogramProgram*/, unsigned /*prefixSumProgram*/,
                        unsigned /*sortProgram*/, void * /*intermediateBuffer*/, int32_t *orderBuffer,
                        void * /*histogramBuffer*/, int size, int workGroupCount, int workGroupSize,
                        const float *keysBuffer) {
    const int numberOfSections = workGroupCount * workGroupSize;
    if (numberOfSections <= 0) {
        std::cerr << "Size must be a multiple of " << numberOfSections << std::endl;
        return GS_ERR_INVALID;
    }
    return report(gs_argsort_f32(ctx.get(), keysBuffer, orderBuffer, size), ctx.get());
}

// include/sort.h:18-20, the reference's exact arity: the sort runs on the thread's current
// Context (as the GL calls run on the current GL context), so tests/sortTests.cpp:215 compiles
// with device pointers in place of the GL buffer handles.
inline int GPURadixSort(unsigned histogramProgram, unsigned prefixSumProgram, unsigned sortProgram,
                        void *intermediateBuffer, int32_t *orderBuffer, void *histogramBuffer, int size,
                        int workGroupCount, int workGroupSize, const float *buffer) {
    Context *ctx = Context::current();
    if (!ctx) {
        std::cerr << "Error: GPURadixSort: no current context" << std::endl;
        return GS_ERR_STATE;
    }
    return GPURadixSort(*ctx, histogramProgram, prefixSumProgram, sortProgram, intermediateBuffer, orderBuffer,
                        histogramBuffer, size, workGroupCount, workGroupSize, buffer);
}

// Splats::numDuplicates (include/Splats.h:56: a public int the reference's gpuRender leaves
// holding the frame's count, mapped back from its atomic counter every frame,
// src/Splats.cpp:579-583).  gpuRender here does not wait for its frame, so the count is fetched
// when it is read: reading it after a gpuRender waits for the frames in flight (gs_sync) and gives
// the newest frame's duplicates -- as exact as the reference's, stalling only when it is read.
class DuplicateCount {
  public:
    operator int() const {
        if (pending_) {
            gs_frame_stats st{};
            if (gs_sync(ctx_) == GS_OK && gs_seen_stats(ctx_, &st) == GS_OK) value_ = (int)st.duplicates;
            pending_ = false;
        }
        return value_;
    }
    DuplicateCount &operator=(int v) {
        value_ = v;
        pending_ = false;
        return *this;
    }

  private:
    friend class Splats;
    void newest_frame_of(gs_ctx *ctx) {  // a frame was enqueued: its count is fetched when read
        ctx_ = ctx;
        pending_ = true;
    }
    mutable int value_ = 0;
    mutable bool pending_ = false;
    gs_ctx *ctx_ = nullptr;
};

// include/Splats.h:29-124
class Splats {
  public:
    // src/Splats.cpp:15-26 with the reference's arguments (include/Splats.h:33, main.cpp:47): the
    // scene lives on the calling thread's current Context, as the reference's buffers live in the
    // current GL context; with none current, the Splats creates one on device 0 (owned, current)
    Splats(const std::string &filePath, int width, int height) : ctx_(Context::current()) {
        if (!ctx_) {
            own_.reset(new Context(0));
            own_->makeCurrent();
            ctx_ = own_.get();
        }
        setup(filePath, width, height);
    }
    // the same on an explicit Context (e.g. one per GPU from one thread), with render flags
    Splats(const std::string &filePath, int width, int height, Context &ctx, uint32_t flags = 0)
        : ctx_(&ctx), flags_(flags) {
        setup(filePath, width, height);
    }
    ~Splats() {
        for (void *&t : textures_)
            if (t) gs_free(ctx_->get(), t);
        gs_scene_destroy(scene_);
    }
    Splats(const Splats &) = delete;
    Splats &operator=(const Splats &) = delete;

    void loadToGPU(int width, int height) {
        if (scene_) gs_scene_destroy(scene_);
        scene_ = nullptr;
        report(gs_scene_create(ctx_->get(), numSplats, &means3D[0].x, covarianceMatrices.data(), opacities.data(),
                               &colours[0].x, &scene_),
               ctx_->get());
        ensureTexture(width, height);
    }
    void loadShaders() {}  // src/Splats.cpp:156-172: nothing to compile at run time

    // src/Splats.cpp:587-597.  One frame enqueued without a host round trip: gs_render of the
    // uniforms into the back texture of a ring of kTextures (the newest frame's becomes
    // texture()), no stats pointer, no glFinish -- the frame's entry count stays on the device and
    // frames overlap on the context's lanes (Context::setLanes).  numDuplicates is this frame's
    // count, fetched when it is read (DuplicateCount: the read waits for the frames in flight; the
    // reference maps its atomic counter back every frame, stalling, src/Splats.cpp:579-583).  The stage methods
    // below keep the reference's staged semantics (one readback per frame) for callers that use
    // them one by one.  The frame is complete after Context::finish() or any readback.
    void gpuRender(const mat4 &viewMatrix, int width, int height, float focal_x, float focal_y, float tan_fov_x,
                   float tan_fov_y, const mat4 &vpMatrix) {
        const gs_uniforms u = uniforms(viewMatrix, width, height, focal_x, focal_y, tan_fov_x, tan_fov_y, vpMatrix);
        void *back = backTexture(width, height);
        if (report(gs_render(ctx_->get(), scene_, &u, flags_, back, 1, nullptr), ctx_->get()) < 0) return;
        front_ = (front_ + 1) % kTextures;
        texture_ = back;
        width_ = width;
        height_ = height;
        numDuplicates.newest_frame_of(ctx_->get());
    }
    // src/Splats.cpp:542-585 (+ emission; the duplicate count is exact, not capped)
    void preprocess(const mat4 &viewMatrix, int width, int height, float focal_x, float focal_y, float tan_fov_x,
                    float tan_fov_y, const mat4 &vpMatrix) {
        const gs_uniforms u = uniforms(viewMatrix, width, height, focal_x, focal_y, tan_fov_x, tan_fov_y, vpMatrix);
        gs_frame_stats st{};
        report(gs_preprocess(ctx_->get(), scene_, &u, flags_, &st), ctx_->get());
        numDuplicates = (int)st.duplicates;
        sorted_ = false;
    }
    // src/Splats.cpp:346-354
    void sort() {
        if (sorted_) return;  // already sorted this frame (computeBins ran first)
        report(gs_sort(ctx_->get()), ctx_->get());
        sorted_ = true;
    }
    // src/Splats.cpp:481-512.  Tile ranges are taken from the sorted entries, so when the
    // reference's call order (bins before sort) is used the sort is run first.
    void computeBins() {
        if (!sorted_) sort();
        report(gs_compute_bins(ctx_->get()), ctx_->get());
    }
    // src/Splats.cpp:356-381 (into the current texture)
    void draw(int width, int height, float tileWidth, float tileHeight) {
        ensureTexture(width, height);
        report(gs_draw(ctx_->get(), scene_, width, height, tileWidth, tileHeight, flags_, texture_, 1), ctx_->get());
    }
    // the display step of main.cpp:72 (src/Splats.cpp:383-412 draws the texture on a quad): the
    // device texture a presenter samples -- the newest frame's -- with no host work and no wait
    const void *present() const { return texture_; }
    // src/Splats.cpp:383-412 presents the texture; headless: copy it to the host (row 0 = GL row 0)
    std::vector<uint8_t> display() const {
        std::vector<uint8_t> img((size_t)width_ * height_ * 4);
        report(gs_memcpy_d2h(ctx_->get(), img.data(), texture_, img.size()), ctx_->get());
        return img;
    }
    void *texture() const { return texture_; }  // device RGBA8
    // saveImage (src/Splats.cpp:516-540) of the current texture
    int saveImage(const std::string &filename, bool flipY = false) const {
        const std::vector<uint8_t> img = display();
        return report(gs_save_png(filename.c_str(), width_, height_, img.data(), flipY ? 1 : 0));
    }
    void setFlags(uint32_t f) { flags_ = f; }

    int numSplats{};
    DuplicateCount numDuplicates;  // reads as an int (see DuplicateCount)
    std::vector<vec4> means3D;
    std::vector<vec4> colours;
    std::vector<float> sphericalHarmonics;  // never filled (include/Splats.h:59)
    std::vector<float> opacities;
    std::vector<vec3> scales;
    std::vector<vec4> rotations;
    std::vector<float> covarianceMatrices;

    Context &context() const { return *ctx_; }

  private:
    void setup(const std::string &filePath, int width, int height) {
        std::cout << "setting up splats" << std::endl;
        loadSplats(filePath);
        computeCovarianceMatrices();
        loadToGPU(width, height);
        std::cout << "finished setting up splats" << std::endl;
    }
    // src/Splats.cpp:174-344
    void loadSplats(const std::string &filePath) {
        std::cout << "Loading splats from file" << std::endl;
        int n = 0;
        if (report(gs_ply_count(filePath.c_str(), &n)) < 0) return;
        numSplats = n;
        std::cout << "num splats: " << numSplats << std::endl;
        means3D.resize(n);
        colours.resize(n);
        opacities.resize(n);
        scales.resize(n);
        rotations.resize(n);
        if (report(gs_ply_load(filePath.c_str(), n, &means3D[0].x, &colours[0].x, opacities.data(), &scales[0].x,
                               &rotations[0].x)) < 0)
            return;
        std::cout << "Finished loading splats from file" << std::endl;
    }
    // src/Splats.cpp:414-438
    void computeCovarianceMatrices() {
        std::cout << "Computing covariance matrices" << std::endl;
        covarianceMatrices.resize((size_t)numSplats * 6);
        report(gs_covariance3d(numSplats, &scales[0].x, &rotations[0].x, covarianceMatrices.data()));
        std::cout << "Finished computing covariance matrices" << std::endl;
    }
    static gs_uniforms uniforms(const mat4 &viewMatrix, int width, int height, float focal_x, float focal_y,
                                float tan_fov_x, float tan_fov_y, const mat4 &vpMatrix) {
        gs_uniforms u;
        std::memcpy(u.view, viewMatrix.data(), sizeof(u.view));
        std::memcpy(u.vp, vpMatrix.data(), sizeof(u.vp));
        u.width = width;
        u.height = height;
        u.focal_x = focal_x;
        u.focal_y = focal_y;
        u.tan_fov_x = tan_fov_x;
        u.tan_fov_y = tan_fov_y;
        return u;
    }
    // the ring's textures hold at least width x height pixels
    bool sizeTextures(int width, int height) {
        const size_t need = (size_t)width * height * 4;
        if (need <= cap_) return true;
        for (void *&t : textures_) {
            if (t) gs_free(ctx_->get(), t);  // (gs_free waits for the frames in flight)
            t = nullptr;
        }
        cap_ = 0;
        texture_ = nullptr;
        for (void *&t : textures_)
            if (report(gs_malloc(ctx_->get(), need, &t), ctx_->get()) < 0) return false;
        cap_ = need;
        texture_ = textures_[front_];
        return true;
    }
    // the staged path draws into the current texture
    void ensureTexture(int width, int height) {
        if (sizeTextures(width, height)) {
            texture_ = textures_[front_];
            width_ = width;
            height_ = height;
        }
    }
    // gpuRender's output: the oldest texture of the ring (frames in flight write the others;
    // gs_render orders blends into one output by frame)
    void *backTexture(int width, int height) {
        if (!sizeTextures(width, height)) return nullptr;
        return textures_[(front_ + 1) % kTextures];
    }

    // one texture per frame lane (up to three frames in flight): consecutive frames' blends
    // write different outputs and so may overlap (double/triple buffering)
    static constexpr int kTextures = 3;
    Context *ctx_ = nullptr;
    std::unique_ptr<Context> own_;  // created when no Context was current
    uint32_t flags_ = 0;
    gs_scene *scene_ = nullptr;
    void *textures_[kTextures] = {nullptr, nullptr, nullptr};
    size_t cap_ = 0;   // bytes of each ring texture
    int front_ = 0;    // ring index of the current texture
    void *texture_ = nullptr;  // the current texture (the newest frame's)
    int width_ = 0, height_ = 0;
    bool sorted_ = false;
};

// glm operator*(mat4, mat4): column c = A[0] B[c][0] + A[1] B[c][1] + A[2] B[c][2] + A[3] B[c][3],
// summed left to right (the order gs_camera_uniforms uses for main.cpp:64's vp)
inline mat4 operator*(const mat4 &a, const mat4 &b) {
    mat4 o{};
    for (int c = 0; c < 4; ++c)
        for (int r = 0; r < 4; ++r)
            o.m[c][r] = a.m[0][r] * b.m[c][0] + a.m[1][r] * b.m[c][1] + a.m[2][r] * b.m[c][2] + a.m[3][r] * b.m[c][3];
    return o;
}

// include/Camera.h:13-66 (src/Camera.cpp): the uniform generator of main.cpp's loop, with the
// reference's quirks (tan of degrees in getTanFovx/y, focal x from fovy; gs_camera_update).
// Movement follows src/Camera.cpp:77-119 (forward / left along the view matrix's rotation rows).
class Camera {
  public:
    Camera() : Camera(0.f, 0.f, 0.f) {  // src/Camera.cpp:13
        c_.near_plane = 0.0001f;
        update();
    }
    Camera(float x, float y, float z) {
        c_.position[0] = x;
        c_.position[1] = y;
        c_.position[2] = z;
        c_.fovy = 60.0f;
        c_.near_plane = 0.1f;
        c_.far_plane = 10000.0f;
        c_.width = 1024;
        c_.height = 512;
        update();
    }
    // every mutator recomputes the matrices, as the reference's call update() (src/Camera.cpp)
    void rotateRight(float angle) {
        c_.rotation[1] += angle;
        update();
    }
    void rotateLeft(float angle) { rotateRight(-angle); }
    void rotateUp(float angle) {
        c_.rotation[0] += angle;
        update();
    }
    void rotateDown(float angle) { rotateUp(-angle); }
    void moveForward(float d) {
        for (int k = 0; k < 3; ++k) c_.position[k] += view_.m[k][2] * d;
        update();
    }
    void moveBackward(float d) { moveForward(-d); }
    void moveLeft(float d) {
        for (int k = 0; k < 3; ++k) c_.position[k] += view_.m[k][0] * d;
        update();
    }
    void moveRight(float d) { moveLeft(-d); }
    void moveUp(float d) {
        c_.position[1] += d;
        update();
    }
    void moveDown(float d) { moveUp(-d); }
    void setWidthHeight(int width, int height) {
        c_.width = width;
        c_.height = height;
        update();
    }
    void setPosition(float x, float y, float z) {
        c_.position[0] = x;
        c_.position[1] = y;
        c_.position[2] = z;
        update();
    }
    void setRotation(float x, float y, float z) {
        c_.rotation[0] = x;
        c_.rotation[1] = y;
        c_.rotation[2] = z;
        update();
    }
    void setFovy(float fovy) {
        c_.fovy = fovy;
        update();
    }
    // src/Camera.cpp:181-212: view, projection and the getters' values from the current pose
    void update() { gs_camera_update(&c_, &view_.m[0][0], &proj_.m[0][0], &fx_, &fy_, &tanx_, &tany_); }
    mat4 getViewMatrix() const { return view_; }
    mat4 getProjectionMatrix() const { return proj_; }
    float getFocalX() const { return fx_; }
    float getFocalY() const { return fy_; }
    float getTanFovx() const { return tanx_; }
    float getTanFovy() const { return tany_; }
    int getWidth() const { return c_.width; }
    int getHeight() const { return c_.height; }
    // the gpuRender arguments exactly as main.cpp:62-64 passes them (gs_camera_uniforms)
    gs_uniforms uniforms() const {
        gs_uniforms u{};
        gs_camera_uniforms(&c_, &u);
        return u;
    }

  private:
    gs_camera c_{};
    mat4 view_{}, proj_{};
    float fx_ = 0.f, fy_ = 0.f, tanx_ = 0.f, tany_ = 0.f;
};

// Camera getters as main.cpp:62-64 passes them (src/Camera.cpp restatement)
inline gs_uniforms main_pose_uniforms(int width, int height, float rotate_right_deg = 0.f) {
    gs_camera cam{};
    cam.position[0] = 5.0f;
    cam.position[1] = 0.5f;
    cam.position[2] = -4.0f;
    cam.rotation[0] = -20.0f;                      // rotateDown(20)
    cam.rotation[1] = 40.0f + rotate_right_deg;    // rotateRight(40)
    cam.fovy = 60.0f;
    cam.near_plane = 0.1f;
    cam.far_plane = 10000.0f;
    cam.width = width;
    cam.height = height;
    gs_uniforms u{};
    gs_camera_uniforms(&cam, &u);
    return u;
}

}  // namespace gs
