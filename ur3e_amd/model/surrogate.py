"""Mesh surrogate for the reference MJCF models.

The reference models (`assets/main.xml:16-42`, `assets/ur3e_2f85.xml:16-37`,
`assets/ur3e_raw.xml:7-13`) reference STL/OBJ meshes that the reference repo
git-ignores (`.gitignore:2-4`): they exist nowhere.  The meshes set two things in
MuJoCo:

* the collision shape of every arm link and every 2F-85 link except the pad
  boxes, and
* the mass/inertia of bodies without an `<inertial>` element (MuJoCo's default
  `inertiafromgeom="auto"` integrates every geom of such a body, visual ones
  included): `robot_base`, `robotiq_base_mount` (`main.xml:152-155`) and the
  two `*_silicone_pad` bodies (`main.xml:197-199, 235-237`).

This module is the documented, NON-REFERENCE replacement.  Every mesh becomes a
box in the mesh-geom's frame.  Boxes are sized to the UR3e/2F-85 link envelopes
implied by the MJCF body offsets; mass is `density(1000) * box volume` per geom,
exactly like MuJoCo would integrate a mesh of that volume.

`collide=False` turns a surrogate into a visual-only geom (contype = conaffinity
= 0).  The 2F-85 four-bar linkage links (driver / coupler / spring_link /
follower) and the base mount get this: without their real shapes, box stand-ins
inside the linkage would generate spurious internal contacts.  All object-side
contact of the gripper goes through the exact pad boxes (`main.xml:81-88`).

Model parity with reference MuJoCo is therefore unpinnable; the
CPU oracle in `oracle/` consumes the same compiled model.
"""

# mesh name -> (half sizes, center in geom frame, collide)
MESH_SURROGATE = {
    # UR3e arm (ur3e/mesh/collision/*.stl)
    "base": ((0.064, 0.064, 0.045), (0.0, 0.0, 0.045), True),
    "shoulder": ((0.045, 0.08, 0.045), (0.0, 0.035, 0.0), True),
    "upperarm": ((0.04, 0.04, 0.15), (0.0, 0.0, 0.122), True),
    "forearm": ((0.035, 0.035, 0.13), (0.0, 0.0, 0.1065), True),
    "wrist1": ((0.032, 0.055, 0.032), (0.0, 0.05, 0.0), True),
    "wrist2": ((0.032, 0.032, 0.048), (0.0, 0.0, 0.04), True),
    "wrist3": ((0.032, 0.022, 0.032), (0.0, 0.06, 0.0), True),
    # Robotiq 2F-85 (2f85/mesh/*.stl, scale 0.001 in the MJCF)
    "gripper_base_mount": ((0.0375, 0.0375, 0.0019), (0.0, 0.0, 0.0019), False),
    "gripper_base": ((0.03, 0.045, 0.0345), (0.0, 0.0, 0.0345), True),
    "gripper_driver": ((0.005, 0.012, 0.01), (0.0, 0.015, 0.0), False),
    "gripper_coupler": ((0.005, 0.004, 0.02), (0.0, 0.003, 0.02), False),
    "gripper_spring_link": ((0.006, 0.02, 0.02), (0.0, 0.018, 0.02), False),
    "gripper_follower": ((0.005, 0.008, 0.015), (0.0, -0.01, 0.012), False),
    "gripper_pad": ((0.011, 0.004, 0.0185), (0.0, -0.0026, 0.0185), False),
    "gripper_silicone_pad": ((0.011, 0.001, 0.0185), (0.0, -0.0075, 0.0185), False),
    "fish": ((0.03, 0.02, 0.055111), (0.0, 0.0, 0.0), False),
}

DENSITY = 1000.0  # MuJoCo default geom density
