/*
 * crt_renderer — command-line front end, drop-in for src/standalone/main.cpp.
 *
 *   crt_renderer [<scene-file>] [<output-file>]            (reference interface, main.cpp:14,28)
 *   crt_renderer [...] [--width W] [--height H] [--max-depth D] [--gi-rays N] [--gpus G | --device K]
 *
 * Same defaults ("../scenes/15-01-conclusion/scene2.crtscene", "output.ppm"),
 * same messages and exit codes (main.cpp:16-33), same timed region (only the
 * render call, main.cpp:37-43: scene upload happens before the timer, the
 * device-to-host copy of the image is inside it like the reference's returned
 * Image), same PPM bytes (crt_image_ppm.cpp).  The flags are additions: the
 * reference CLI always uses default RendererSettings and the file's size.
 *
 * Like the reference's render_image, which spans every hardware thread
 * (crt_renderer.cpp:176-196), the render may span several GPUs: by default as
 * many as the frame's size pays for (crt_hip_scene_create_auto: one GPU for a
 * short frame, all of them for a GI or very large one; CRT_HIP_GPUS=N sets
 * the count); --gpus G takes devices 0..G-1, --device K one device.
 */
#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "../../../include/crt_hip.h"

static std::string quoted(const char *p) {   /* std::filesystem::path's operator<< quotes */
    std::string s = "\"";
    for (const char *c = p; *c; ++c) {
        if (*c == '"' || *c == '\\') s += '\\';
        s += *c;
    }
    return s + "\"";
}

int main(int argc, char *argv[]) {
    std::vector<const char *> pos;
    int width = -1, height = -1, device = -1, gpus = 0;
    long max_depth = -1, gi_rays = -1;
    for (int i = 1; i < argc; ++i) {
        const std::string a = argv[i];
        auto next = [&](long &v) {
            if (i + 1 >= argc) { std::fprintf(stderr, "Error: %s needs a value\n", a.c_str()); std::exit(2); }
            v = std::strtol(argv[++i], nullptr, 10);
        };
        long v;
        if (a == "--width") { next(v); width = (int)v; }
        else if (a == "--height") { next(v); height = (int)v; }
        else if (a == "--max-depth") { next(max_depth); }
        else if (a == "--gi-rays") { next(gi_rays); }
        else if (a == "--device") { next(v); device = (int)v; }
        else if (a == "--gpus") { next(v); gpus = (int)v; }
        else if (a == "--help" || a == "-h") {
            std::printf("usage: crt_renderer [<scene-file>] [<output-file>] [--width W] [--height H] "
                        "[--max-depth D] [--gi-rays N] [--gpus G | --device K]\n");
            return 0;
        } else pos.push_back(argv[i]);
    }
    const char *input = pos.size() > 0 ? pos[0] : "../scenes/15-01-conclusion/scene2.crtscene";
    const char *output = pos.size() > 1 ? pos[1] : "output.ppm";

    std::FILE *probe = std::fopen(input, "rb");
    if (!probe) {
        std::fprintf(stderr, "Error: Could not open input file: %s\n", quoted(input).c_str());
        return 1;
    }
    std::fclose(probe);
    crt_scene_file *sf = nullptr;
    if (crt_scene_file_load(input, &sf) != CRT_OK) {
        std::fprintf(stderr, "Error: Could not parse JSON file: %s\n", quoted(input).c_str());
        return 1;
    }
    const crt_scene_desc *desc = crt_scene_file_desc(sf);
    if (width > 0 || height > 0)
        crt_scene_file_set_resolution(sf, width > 0 ? width : desc->camera.width,
                                      height > 0 ? height : desc->camera.height);

    std::FILE *out = std::fopen(output, "wb");
    if (!out) {
        std::fprintf(stderr, "Error: Could not open output file: %s\n", output);
        crt_scene_file_destroy(sf);
        return 1;
    }
    std::fclose(out);

    crt_renderer_settings settings;
    crt_renderer_settings_default(&settings);
    if (max_depth >= 0) settings.max_ray_depth = (uint32_t)max_depth;
    if (gi_rays >= 0) settings.diffuse_reflection_ray_count = (uint32_t)gi_rays;

    crt_hip_scene *scene = nullptr;
    const uint64_t mask = gpus >= 64 ? ~0ull : (1ull << std::max(gpus, 0)) - 1ull;
    const int crc = device >= 0 ? crt_hip_scene_create(desc, device, &scene)
                    : gpus > 0  ? crt_hip_scene_create_mask(desc, mask, CRT_SCENE_TREE_AUTO, &scene)
                                : crt_hip_scene_create_auto(desc, &settings, CRT_SCENE_TREE_AUTO, &scene);
    if (crc != CRT_OK) {
        std::fprintf(stderr, "Error: %s\n", crt_hip_last_error());
        crt_scene_file_destroy(sf);
        return 1;
    }
    const int W = desc->camera.width, H = desc->camera.height;
    std::vector<float> image((size_t)W * H * 3);

    const auto start = std::chrono::high_resolution_clock::now();
    const int rc = crt_hip_render(scene, &settings, image.data(), nullptr);
    const auto stop = std::chrono::high_resolution_clock::now();
    if (rc != CRT_OK) {
        std::fprintf(stderr, "Error: %s\n", crt_hip_last_error());
        crt_hip_scene_destroy(scene);
        crt_scene_file_destroy(sf);
        return 1;
    }
    const long long us = std::chrono::duration_cast<std::chrono::microseconds>(stop - start).count();
    std::printf("Execution time: %Lg seconds.\n", (long double)us / 1000000.0L);

    int wrc = crt_write_ppm(output, image.data(), W, H, 255);
    crt_hip_scene_destroy(scene);
    crt_scene_file_destroy(sf);
    if (wrc != CRT_OK) {
        std::fprintf(stderr, "Error: %s\n", crt_hip_last_error());
        return 1;
    }
    return 0;
}
