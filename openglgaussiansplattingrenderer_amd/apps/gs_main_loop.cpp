// gs_main_loop -- the reference's frame loop (main.cpp:40-89) through the kept C++ API
// (include/gsplat_splats.hpp): Camera(5, 0.5, -4), rotateDown(20), rotateRight(40), the
// three-argument Splats(path, W, H), then per frame the pose update, Splats::gpuRender with
// main.cpp:62-64's arguments and the display step (Splats::present: the texture a presenter
// samples).  Headless: no window, no input (a static pose, as main.cpp without key presses, or
// rotateRight(turn) per frame).  Two loops over the same poses, wall clock:
//   serial -- one frame at a time, as main.cpp blocks on the frame's GL_TIMESTAMP query
//             (main.cpp:84-87): Context::finish() after each frame;
//   ahead  -- frames enqueued ahead on the context's lanes, finish() after the last.
// Their last images must be identical (printed).  One JSON line on stdout.
// usage: gs_main_loop <scene.ply> <W> <H> <frames> <warmup> <lanes> [turn_deg_per_frame [out_rgba8.bin]]
// (out_rgba8.bin: the last frame's image, row y = GL row y, for the parity test)
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <iostream>
#include <vector>

#include "gsplat_splats.hpp"

int main(int argc, char **argv) {
    if (argc < 7) {
        std::cerr << "usage: gs_main_loop <scene.ply> <W> <H> <frames> <warmup> <lanes> [turn]\n";
        return 2;
    }
    const char *path = argv[1];
    const int W = std::atoi(argv[2]), H = std::atoi(argv[3]);
    const int frames = std::atoi(argv[4]), warmup = std::atoi(argv[5]), lanes = std::atoi(argv[6]);
    const float turn = argc > 7 ? (float)std::atof(argv[7]) : 0.0f;
    gs::Context ctx(0);
    if (!ctx.get()) return 3;
    if (ctx.setLanes(lanes) < 0) return 3;
    // one timestamp per frame, as main.cpp:52-58's GL_TIMESTAMP queries (the library's default
    // times every stage boundary, whose events idle the stream a few microseconds each)
    if (gs_timing_enable(ctx.get(), GS_TIMING_FRAME) != GS_OK) return 3;
    // main.cpp:40-45
    gs::Camera camera(5.0f, 0.5f, -4.0f);
    camera.rotateDown(20.0f);
    camera.rotateRight(40.0f);
    camera.setWidthHeight(W, H);
    camera.update();
    const auto tl0 = std::chrono::steady_clock::now();
    gs::Splats splats(path, camera.getWidth(), camera.getHeight());  // main.cpp:47
    const double load_s = std::chrono::duration<double>(std::chrono::steady_clock::now() - tl0).count();
    if (splats.numSplats <= 0) return 4;
    // main.cpp:62-64's arguments must be gs_camera_uniforms' (the tan swap, vp = P * V)
    {
        const gs_uniforms a = camera.uniforms();
        const gs::mat4 vp = camera.getProjectionMatrix() * camera.getViewMatrix();
        if (std::memcmp(a.vp, vp.data(), sizeof(a.vp)) != 0 || a.tan_fov_x != camera.getTanFovy()) {
            std::cerr << "FAILED: camera getters differ from gs_camera_uniforms\n";
            return 5;
        }
    }
    const void *shown = nullptr;
    auto frame = [&](int k) {
        if (turn != 0.0f && k > 0) camera.rotateRight(turn);  // (camera.getInput, main.cpp:76)
        splats.gpuRender(camera.getViewMatrix(), camera.getWidth(), camera.getHeight(), camera.getFocalX(),
                         camera.getFocalY(), camera.getTanFovy(), camera.getTanFovx(),
                         camera.getProjectionMatrix() * camera.getViewMatrix());
        shown = splats.present();  // splats.display() (main.cpp:72)
    };
    auto run = [&](bool serial, std::vector<uint8_t> &last) {
        camera.setRotation(-20.0f, 40.0f, 0.0f);  // the same poses in both loops
        for (int k = 0; k < warmup; ++k) frame(0);
        ctx.finish();
        camera.setRotation(-20.0f, 40.0f, 0.0f);
        const auto t0 = std::chrono::steady_clock::now();
        for (int k = 0; k < frames; ++k) {
            frame(k);
            if (serial) ctx.finish();  // main.cpp:84-87 waits for the frame's end timestamp
        }
        ctx.finish();
        const double s = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
        last = splats.display();
        return s;
    };
    std::vector<uint8_t> img_serial, img_ahead;
    const double s_serial = run(true, img_serial);
    const double s_ahead = run(false, img_ahead);
    const bool same = img_serial == img_ahead;
    if (argc > 8) {
        std::FILE *f = std::fopen(argv[8], "wb");
        if (!f || std::fwrite(img_ahead.data(), 1, img_ahead.size(), f) != img_ahead.size()) return 6;
        std::fclose(f);
    }
    // numDuplicates read after the loops: the newest frame's (the last pose), as the reference's
    // gpuRender leaves it (src/Splats.cpp:579-583)
    const int dups = splats.numDuplicates;
    gs_frame_stats st{};
    gs_last_stats(ctx.get(), &st);
    std::printf("{\"frames\": %d, \"warmup\": %d, \"lanes\": %d, \"turn_deg_per_frame\": %g, \"splats\": %d, "
                "\"E\": %lld, \"numDuplicates\": %d, \"serial_fps\": %.3f, \"serial_ms_per_frame\": %.4f, "
                "\"ahead_fps\": %.3f, \"ahead_ms_per_frame\": %.4f, \"last_images_identical\": %s, \"load_s\": %.3f, "
                "\"presented\": %s}\n",
                frames, warmup, lanes, turn, splats.numSplats, (long long)st.entries, dups,
                frames / s_serial, s_serial / frames * 1e3, frames / s_ahead, s_ahead / frames * 1e3,
                same ? "true" : "false", load_s, shown ? "true" : "false");
    return same ? 0 : 1;
}
