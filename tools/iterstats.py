import sys
sys.path.insert(0, ".")
import torch  # noqa
import wpt_loader
w = wpt_loader.load(); itf = w.interface
W, H, spp = 1920, 1080, 8
itf.init(W, H, 2, *w.scenes.scene_camera(2))
itf.store_mesh(1, w.scenes.triangle_cloud(100000))
itf.update_settings(1, 1, 0, 0, 0)
itf.set_render_options(8, 0xBABABEBE, 1 << 27)
itf.set_counting(True)
itf.compute(W * H * spp); itf.sync()
st = itf.stats()
live = st["ext_live_iters"]
print("live iters", live, "rays", st["rays"], "steps/ray", live / st["rays"])
for k, name in (("stamp_expand", "leaf-only iterations"), ("stamp_leaf", "far leaf kept pending"), ("stamp_pop", "pop resumed a leaf")):
    print(name, round(st[k] * 64 / live, 4))
