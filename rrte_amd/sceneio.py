"""SceneIR dump / load for repro (include/rrte_hip.h rrte_hip_scene_dump / _load, format in
rrte_amd/csrc/scene_io.hip): one frame's lowered scene and render parameters in a self-checking file,
replayable bit for bit on the device or on the CPU oracle.  `RRTE_DUMP_SCENE=<path>` makes every render
entry point of the library write the frame it is given to <path> before rendering it."""
from __future__ import annotations

import ctypes as C

from . import abi


def dump(scene_ref, params, path: str) -> None:
    """Writes the scene (a ctypes reference to an abi.SceneIR, e.g. LoweredScene.ref()) and the render
    parameters (abi.RenderParams) to `path`."""
    lib = abi.load()
    st = lib.rrte_hip_scene_dump(scene_ref, C.byref(params), str(path).encode())
    if st != abi.RRTE_OK:
        raise abi.RrteError(st, f"rrte_hip_scene_dump({path}) failed")


class LoadedScene:
    """A dumped frame: `.ir` (abi.SceneIR) and `.params` (abi.RenderParams); the arrays live in the
    library's storage until close() (or garbage collection)."""

    def __init__(self, path: str):
        self._lib = abi.load()
        self.ir = abi.SceneIR()
        self.params = abi.RenderParams()
        self._storage = C.c_void_p()
        st = self._lib.rrte_hip_scene_load(str(path).encode(), C.byref(self.ir), C.byref(self.params),
                                           C.byref(self._storage))
        if st != abi.RRTE_OK:
            raise abi.RrteError(st, f"rrte_hip_scene_load({path}): missing, truncated, altered or another ABI")

    def ref(self):
        return C.byref(self.ir)

    def close(self):
        if self._storage:
            self._lib.rrte_hip_scene_free(self._storage)
            self._storage = C.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def load(path: str) -> LoadedScene:
    return LoadedScene(path)
