// yrt_raytrace -- drop-in for the reference's bin/raytrace (main, src/raytrace.cpp:256-287):
//
//     yrt_raytrace [-r RES] [-s SAMPLES] [-a AMBIENT] [-o OUT.png|OUT.hdr] scene.obj
//
// same options, defaults (720, 1, 0.1, out.png), messages and output file as the
// reference, over the C++ mirror in include/yrt_raytrace.hpp. Extra options (not in
// the reference): --device N, --width W, --max-depth D, --algorithm
// wavefront|megakernel|wavefront_lane, --time (print GPU time and Mrays/s).
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>

#include "yrt_raytrace.hpp"

namespace {

[[noreturn]] void usage(const char* msg) {
    if (msg) fprintf(stderr, "error: %s\n", msg);
    fprintf(stderr,
            "usage: yrt_raytrace [options] scenein\n"
            "  -r, --resolution N   vertical resolution [720]\n"
            "  -s, --samples N      per-pixel samples per axis (N*N rays per pixel) [1]\n"
            "  -a, --ambient F      ambient color [0.1]\n"
            "  -o, --output FILE    output image (.png tonemapped, .hdr float) [out.png]\n"
            "  --device N           GPU index [0]\n"
            "  --gpus N             split the frame over N GPUs from --device on [1]\n"
            "  --width N            explicit width (default round(aspect * resolution))\n"
            "  --max-depth N        cap on reflection depth [16]\n"
            "  --algorithm NAME     wavefront | megakernel | wavefront_lane [wavefront]\n"
            "  --time               print render time and Mrays/s\n");
    exit(msg ? 1 : 0);
}

int parse_int(const char* s, const char* opt) {
    char* end = nullptr;
    long v = strtol(s, &end, 10);
    if (!*s || *end) usage((std::string("bad value for ") + opt).c_str());
    return (int)v;
}

}  // namespace

int main(int argc, char** argv) {
    int resolution = 720, samples = 1, device = 0, gpus = 1, width = 0, max_depth = 16, algorithm = YRT_ALGO_WAVEFRONT;
    float amb = 0.1f;
    bool timing = false;
    std::string out = "out.png", scenein;
    for (int k = 1; k < argc; k++) {
        std::string a = argv[k];
        auto val = [&]() -> const char* {
            if (k + 1 >= argc) usage(("missing value for " + a).c_str());
            return argv[++k];
        };
        if (a == "-r" || a == "--resolution") resolution = parse_int(val(), "-r");
        else if (a == "-s" || a == "--samples") samples = parse_int(val(), "-s");
        else if (a == "-a" || a == "--ambient") amb = strtof(val(), nullptr);
        else if (a == "-o" || a == "--output") out = val();
        else if (a == "--device") device = parse_int(val(), "--device");
        else if (a == "--gpus") gpus = parse_int(val(), "--gpus");
        else if (a == "--width") width = parse_int(val(), "--width");
        else if (a == "--max-depth") max_depth = parse_int(val(), "--max-depth");
        else if (a == "--algorithm") {
            std::string n = val();
            if (n == "wavefront") algorithm = YRT_ALGO_WAVEFRONT;
            else if (n == "megakernel") algorithm = YRT_ALGO_MEGAKERNEL;
            else if (n == "wavefront_lane") algorithm = YRT_ALGO_WAVEFRONT_LANE;
            else usage("unknown --algorithm");
        } else if (a == "--time") timing = true;
        else if (a == "-h" || a == "--help") usage(nullptr);
        else if (!a.empty() && a[0] == '-') usage(("unknown option " + a).c_str());
        else if (scenein.empty()) scenein = a;
        else usage("too many arguments");
    }
    if (scenein.empty()) scenein = "scene.obj";  // the reference's default positional value
    if (gpus < 1) usage("--gpus must be >= 1");
    try {
        printf("loading scene %s\n", scenein.c_str());
        auto scn = yrt_cpp::load_scene(scenein);
        printf("creating bvh\n");
        yrt_cpp::build_bvh(scn, false);
        scn->device = device;
        scn->gpus = gpus;
        scn->params.width = width;
        scn->params.max_depth = max_depth;
        scn->params.algorithm = algorithm;
        printf("tracing scene\n");
        if (timing) yrt_cpp::raytrace(scn, {amb, amb, amb}, resolution, samples);  // upload + warm up
        auto t0 = std::chrono::steady_clock::now();
        auto hdr = yrt_cpp::raytrace(scn, {amb, amb, amb}, resolution, samples);
        auto t1 = std::chrono::steady_clock::now();
        if (timing) {
            const yrt_stats st = yrt_cpp::last_stats(scn);
            double s = std::chrono::duration<double>(t1 - t0).count();
            printf("render %dx%d x %d spp on %d GPU(s): %.3f ms (incl. copy to host), %llu rays, %.1f Mrays/s "
                   "(%llu shadow rays with a zero light term answered without a walk)\n",
                   hdr.width, hdr.height, samples * samples, gpus, s * 1e3, st.rays, st.rays / s / 1e6,
                   st.shadow_rays_culled);
        }
        printf("saving image %s\n", out.c_str());
        yrt_cpp::save_hdr_or_ldr(out, hdr);
    } catch (const yrt_cpp::error& e) {
        fprintf(stderr, "%s\n", e.what());
        return 1;
    }
    return 0;
}
