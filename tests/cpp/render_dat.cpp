// tests/cpp/render_dat.cpp -- TEST PROGRAM: GpuPathRenderer::Render's call sequence
// (integration/gpupathrenderer.cpp:37-92) without the reference's headers, so the GPU box (which
// has no /root/reference) runs the binding's exact C-ABI usage:
//   pbrtgpu_context_create per device -> pbrthost_load -> pbrthost_flat -> pbrtgpu_scene_upload
//   per device -> pbrtgpu_render_multi (16x16 interleaved tiles, host gather) ->
//   pbrthost_write_dat_scene -> pbrtgpu_context_destroy / pbrthost_free.
// The only difference: the resolution / spp / maxdepth / seed overrides a test fixture needs
// (the binding keeps the scene file's, -1).  tests/test_binding.py compares the .dat with the
// reference film's own (tests/golden/killeroo_dat_40x32s4.npz).
// Usage: render_dat SCENE OUT.dat XRES YRES SPP [NGPU [SLICES [gpusetup]]]
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>
#include "pbrthost.h"
#include "pbrtgpu.h"

int main(int argc, char **argv) {
    if (argc < 6) {
        fprintf(stderr, "usage: %s SCENE OUT.dat XRES YRES SPP [NGPU [SLICES [gpusetup]]]\n", argv[0]);
        return 2;
    }
    const int ngpu = argc > 6 ? atoi(argv[6]) : 0, slices = argc > 7 ? atoi(argv[7]) : 1;
    const bool gpuSetup = argc > 8 && !strcmp(argv[8], "gpusetup");
    int ndev = pbrtgpu_device_count();
    if (ndev <= 0) {
        fprintf(stderr, "render_dat: no device\n");
        return 3;
    }
    int n = ngpu > 0 ? (ngpu < ndev ? ngpu : ndev) : ndev;
    pbrthost_overrides ov = {PBRTHOST_ABI_VERSION, atoi(argv[3]), atoi(argv[4]), atoi(argv[5]), 5, 0, 0u, -1, -1, -1, -1, 0,
                             -1};
    std::vector<pbrtgpu_ctx *> ctx(n, (pbrtgpu_ctx *)NULL);
    int status = 0;
    for (int d = 0; d < n && status == 0; ++d) status = pbrtgpu_context_create(d, &ctx[d]);
    pbrthost_scene *hs = NULL;
    char err[1024];
    if (status == 0) {
        if (gpuSetup) pbrthost_set_loop_subdivider(pbrtgpu_loop_subdivide_hook, ctx[0]);
        status = pbrthost_load(argv[1], &ov, &hs, err, sizeof(err));
        if (gpuSetup) pbrthost_set_loop_subdivider(NULL, NULL);
        if (status != 0) fprintf(stderr, "render_dat: %s\n", err);
    } else fprintf(stderr, "render_dat: %s\n", pbrtgpu_last_error());
    if (status == 0) {
        pbrtgpu_flat_scene fs;
        pbrthost_flat(hs, &fs);
        const int W = fs.camera.px_count, H = fs.camera.py_count, N = fs.n_bands;
        for (int d = 0; d < n && status == 0; ++d) status = pbrtgpu_scene_upload(ctx[d], &fs);
        std::vector<float> film((size_t)W * H * N, 0.f);
        if (status == 0) {
            pbrtgpu_render_desc rd = {0, fs.spp, 16, 16, 0, {0, 0, 0}};
            status = pbrtgpu_render_multi(ctx.data(), n, &rd, NULL, 0, slices, film.data(), (int64_t)film.size(), NULL);
        }
        if (status != 0) fprintf(stderr, "render_dat: %s\n", pbrtgpu_last_error());
        if (status == 0 && pbrthost_write_dat_scene(hs, argv[2], film.data(), NULL) != 0) {
            fprintf(stderr, "render_dat: cannot write %s\n", argv[2]);
            status = PBRTGPU_E_INVALID;
        }
    }
    for (int d = 0; d < n; ++d)
        if (ctx[d]) pbrtgpu_context_destroy(ctx[d]);
    if (hs) pbrthost_free(hs);
    fprintf(stderr, "render_dat: status %d\n", status);
    return status == 0 ? 0 : 1;
}
