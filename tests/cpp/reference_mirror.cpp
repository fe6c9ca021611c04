// C++ mirror of the reference's own gtest cases (no gtest in this image: plain asserts),
// written against the drop-in facade include/gsplat_splats.hpp:
//   SortTest.SortTest        tests/sortTests.cpp:127-253
//   SplatsTest.LoadSimplePly tests/plyParseTests.cpp:105-109
//   + one C1 frame through Splats::gpuRender (main.cpp:62-64 uniforms), RGBA8 written to a
//     file for the Python side to compare with the golden fixture.
// usage: reference_mirror <testSingleItem.ply> <out_rgba8.bin>
#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <iostream>
#include <thread>
#include <vector>

#include "gsplat_splats.hpp"

#define EXPECT(c)                                                                    \
    do {                                                                             \
        if (!(c)) {                                                                  \
            std::cerr << "FAILED: " #c " (" << __FILE__ << ":" << __LINE__ << ")\n"; \
            return 1;                                                                \
        }                                                                            \
    } while (0)

// src/utils.cpp:49-63
static std::vector<float> createRandomNumbersFloat(int size) {
    srand(20);
    std::vector<float> r(size);
    for (int i = 0; i < size; i++) {
        int random = rand() % 255;
        r[i] = (float)rand() / RAND_MAX + random + 0.5f;
    }
    return r;
}

static int sort_test(gs::Context &ctx) {
    unsigned hp, sp, up;
    gs::createAndLinkSortAndHistogramShaders(hp, sp, up);
    std::vector<float> randomNumbers = createRandomNumbersFloat(32 * 16 * 10000 - 7);
    const int size = (int)randomNumbers.size();
    std::vector<int32_t> ascending(size);
    for (int i = 0; i < size; i++) ascending[i] = i;
    void *keys = nullptr, *order = nullptr;
    EXPECT(gs_malloc(ctx.get(), size * 4, &keys) == GS_OK);
    EXPECT(gs_malloc(ctx.get(), size * 4, &order) == GS_OK);
    EXPECT(gs_memcpy_h2d(ctx.get(), keys, randomNumbers.data(), size * 4) == GS_OK);
    EXPECT(gs_memcpy_h2d(ctx.get(), order, ascending.data(), size * 4) == GS_OK);
    auto t0 = std::chrono::steady_clock::now();
    // sortTests.cpp:215, the reference's 10 arguments (the thread's current context)
    EXPECT(gs::GPURadixSort(hp, up, sp, nullptr, (int32_t *)order, nullptr, size, 16, 32, (const float *)keys) ==
           GS_OK);
    ctx.finish();
    auto t1 = std::chrono::steady_clock::now();
    std::cout << "GPU sort took " << std::chrono::duration<double>(t1 - t0).count() << " seconds" << std::endl;
    std::vector<float> copy(randomNumbers);
    std::sort(randomNumbers.begin(), randomNumbers.end());
    std::vector<int32_t> out(size);
    EXPECT(gs_memcpy_d2h(ctx.get(), out.data(), order, size * 4) == GS_OK);
    for (int i = 1; i < size; i++) {
        EXPECT(copy[out[i]] >= copy[out[i - 1]]);   // sortTests.cpp:241
        EXPECT(copy[out[i]] == randomNumbers[i]);   // sortTests.cpp:242
    }
    // stability (the reference only checks the key sequence): equal keys keep input order
    for (int i = 1; i < size; i++)
        if (copy[out[i]] == copy[out[i - 1]]) EXPECT(out[i] > out[i - 1]);
    std::cout << "Successfully sorted " << size << " numbers" << std::endl;
    gs_free(ctx.get(), keys);
    gs_free(ctx.get(), order);
    return 0;
}

int main(int argc, char **argv) {
    if (argc < 3) {
        std::cerr << "usage: reference_mirror <testSingleItem.ply> <out_rgba8.bin>\n";
        return 2;
    }
    gs::Context ctx(0);
    if (!ctx.get()) return 3;
    if (sort_test(ctx)) return 1;
    {
        // plyParseTests.cpp:105-109 and main.cpp:47: the reference's three arguments (the scene
        // goes to the current Context, as the reference's buffers go to the current GL context)
        gs::Splats splats(argv[1], 100, 100);
        EXPECT(splats.numSplats == 1);
        EXPECT(&splats.context() == &ctx);
    }
    {
        gs::Splats splats(argv[1], 256, 256);
        const gs_uniforms u = gs::main_pose_uniforms(256, 256);
        gs::mat4 view, vp;
        std::memcpy(view.m, u.view, sizeof(view.m));
        std::memcpy(vp.m, u.vp, sizeof(vp.m));
        splats.gpuRender(view, 256, 256, u.focal_x, u.focal_y, u.tan_fov_x, u.tan_fov_y, vp);
        const std::vector<uint8_t> img = splats.display();
        std::ofstream(argv[2], std::ios::binary).write((const char *)img.data(), (std::streamsize)img.size());
        std::cout << "rendered C1: duplicates " << splats.numDuplicates << std::endl;
        // numDuplicates after gpuRender is that frame's count: the staged preprocess of the same
        // pose (src/Splats.cpp:542-585's readback) gives the same
        const int d_frame = splats.numDuplicates;
        splats.preprocess(view, 256, 256, u.focal_x, u.focal_y, u.tan_fov_x, u.tan_fov_y, vp);
        EXPECT(d_frame == splats.numDuplicates);
    }
    {  // a Context made current here and destroyed on another thread is no longer current here
        gs::Context *other = new gs::Context(0);
        other->makeCurrent();
        EXPECT(gs::Context::current() == other);
        std::thread([other] { delete other; }).join();
        EXPECT(gs::Context::current() == nullptr);
        EXPECT(gs::GPURadixSort(1u, 3u, 2u, nullptr, nullptr, nullptr, 0, 16, 32, nullptr) == GS_ERR_STATE);
        {  // no Context current: the three-argument Splats creates (and makes current) its own
            gs::Splats own(argv[1], 64, 64);
            EXPECT(own.numSplats == 1);
            EXPECT(gs::Context::current() == &own.context() && &own.context() != &ctx);
        }
        EXPECT(gs::Context::current() == nullptr);
        ctx.makeCurrent();
        EXPECT(gs::Context::current() == &ctx);
    }
    std::cout << "ALL PASSED" << std::endl;
    return 0;
}
