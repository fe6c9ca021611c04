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
        if (texture_) gs_free(ctx_->get(), texture_);
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

    // src/Splats.cpp:587-597
    void gpuRender(const mat4 &viewMatrix, int width, int height, float focal_x, float focal_y, float tan_fov_x,
                   float tan_fov_y, const mat4 &vpMatrix) {
        preprocess(viewMatrix, width, height, focal_x, focal_y, tan_fov_x, tan_fov_y, vpMatrix);
        computeBins();
        sort();
        ctx_->finish();
        draw(width, height, float(width) / 16.f, float(height) / 16.f);
    }
    // src/Splats.cpp:542-585 (+ emission; the duplicate count is exact, not capped)
    void preprocess(const mat4 &viewMatrix, int width, int height, float focal_x, float focal_y, float tan_fov_x,
                    float tan_fov_y, const mat4 &vpMatrix) {
        gs_uniforms u;
        std::memcpy(u.view, viewMatrix.data(), sizeof(u.view));
        std::memcpy(u.vp, vpMatrix.data(), sizeof(u.vp));
        u.width = width;
        u.height = height;
        u.focal_x = focal_x;
        u.focal_y = focal_y;
        u.tan_fov_x = tan_fov_x;
        u.tan_fov_y = tan_fov_y;
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
    // src/Splats.cpp:356-381
    void draw(int width, int height, float tileWidth, float tileHeight) {
        ensureTexture(width, height);
        report(gs_draw(ctx_->get(), scene_, width, height, tileWidth, tileHeight, flags_, texture_, 1), ctx_->get());
    }
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
    int numDuplicates{};
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
    void ensureTexture(int width, int height) {
        if (texture_ && (size_t)width * height <= (size_t)width_ * height_) {
            width_ = width;
            height_ = height;
            return;
        }
        if (texture_) gs_free(ctx_->get(), texture_);
        texture_ = nullptr;
        report(gs_malloc(ctx_->get(), (size_t)width * height * 4, &texture_), ctx_->get());
        width_ = width;
        height_ = height;
    }

    Context *ctx_ = nullptr;
    std::unique_ptr<Context> own_;  // created when no Context was current
    uint32_t flags_ = 0;
    gs_scene *scene_ = nullptr;
    void *texture_ = nullptr;
    int width_ = 0, height_ = 0;
    bool sorted_ = false;
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
