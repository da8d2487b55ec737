"""rrte_amd — MI355X-native replacement for rrte-renderer's per-pixel ray->scene loop.

The product is librrte_hip.so (C ABI: include/rrte_hip.h; HIP kernels for
gfx950 in rrte_amd/csrc/).  This package mirrors the reference's renderer API
(Melthizar/RRTE crates/rrte-renderer) on top of that ABI.
"""
from .math import Color, Transform, to_radians, vec3  # noqa: F401
from .renderer import (AmbientLight, BendDeformer, Camera, Capsule, ChainDeformer, Cone, Context,  # noqa: F401
                       CSGComposite, Cube, Cylinder, DeformedSDF, DielectricMaterial, DirectionalLight,
                       EmissiveMaterial, LambertianMaterial, LoweredScene, Material, MetalMaterial,
                       NoiseDeformer, Plane, PointLight, Raytracer, RaytracerConfig, SceneObject, SDF,
                       SDFBox, SDFCapsule, SDFCone, SDFCylinder, SDFEllipsoid, SDFObject, SDFPrism, SDFRing,
                       SDFSphere, SDFTorus, SDFTube, Sphere, SpotLight, TaperDeformer, Triangle,
                       TwistDeformer, WaveDeformer)

from .mesh import Mesh, load_scene_asset  # noqa: F401,E402

__version__ = "0.1.0"
