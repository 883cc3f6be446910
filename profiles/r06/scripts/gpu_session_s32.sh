set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -c "
import wpt_loader
pkg = wpt_loader.load(); itf = pkg.interface
W, H = 3840, 2160
itf.set_option('defaults', 0); itf.set_option('log', 1)
itf.init(W, H, 2, *pkg.scenes.scene_camera(2)); itf.store_mesh(1, pkg.scenes.triangle_cloud(100000))
itf.update_settings(2, 2, 1, 1, 0); itf.set_render_options(8, 0xBABABEBE, 0)
itf.compute(W * H * 80)
print(itf.stats()['stock_traced'])
itf.shutdown()
" > gpurun_out/s32_out.txt 2> gpurun_out/s32_log.txt || { echo FAIL; tail -5 gpurun_out/s32_log.txt; exit 1; }
cat gpurun_out/s32_out.txt; grep "refill id" gpurun_out/s32_log.txt | awk '{print \$5}' | sort -t= -k2 -n | tail -3
timeout -k 10 400 python -u -m pytest tests/test_gpu_stock_4k.py -x -q --timeout 300 --timeout-method thread > gpurun_out/s32_4k.log 2>&1 || { echo TESTFAIL; grep -E "^FAILED|^E " gpurun_out/s32_4k.log | head; exit 1; }
tail -1 gpurun_out/s32_4k.log
