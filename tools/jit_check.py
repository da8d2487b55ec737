import sys; sys.path.insert(0, __import__("os").path.dirname(__import__("os").path.dirname(__import__("os").path.abspath(__file__))))
import ctypes as C, os, sys
from rrte_amd import abi, scenes, LoweredScene
name = sys.argv[1] if len(sys.argv) > 1 else "sdf_showcase"
objs, lights, cam, cfg = getattr(scenes, name)(1920,1080)
sc=LoweredScene(objs,lights,cam)
buf=C.create_string_buffer(20000)
st=abi.load().rrte_hip_jit_check(sc.ref(), 1, buf, 20000)
print("status", st); print(buf.value.decode()[:3000])
