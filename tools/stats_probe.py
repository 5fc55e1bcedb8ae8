"""One cfg2 render with the device counters on (rt_set_stats): the counts and the k_trace byte model split by record kind."""
import sys, os, json
sys.path.insert(0, 'sycl-ray-tracing_amd'); sys.path.insert(0, 'tools'); sys.path.insert(0, '.')
import bench, rt_amd
P, sky, cam17 = bench.build_inputs("cfg2")
_, _, _, W, H, spp, nb, _ = bench.CONFIGS["cfg2"]
rk = rt_amd.RenderKernel(W, H, spp, nb, rt_amd.Image(W, H), P.triangles, P.materials, P.emissive_triangle_indices,
                         P.material_indices, None, rt_amd.BVH(P.triangles), rt_amd.Image.from_rgb(sky), None, device=0)
rk.set_camera(rt_amd.Camera(cam17[:16], cam17[16]))
rk.set_stats(True)
rk.render()
st = rk.stats()
st = {k: int(v) for k, v in st.items()}
b = bench.BYTES
parts = {"box": b["box"] * (st.get("vol", 0) + st.get("any_vol", 0)), "tri": b["tri"] * (st.get("tri", 0) + st.get("any_tri", 0)),
         "verify": b["verify"] * st.get("verify", 0), "ray": b["ray"] * (st.get("rays", 0) + st.get("any_rays", 0))}
print(json.dumps({"stats": st, "bytes": parts}))
