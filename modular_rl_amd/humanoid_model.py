"""Humanoid-v2's model (gym's humanoid.xml) as tables, and its compiled mass properties.

The reference builds Humanoid-v2 with ``gym.envs.make`` (`run_pg.py:85`,
`experiments/battery-trpo.yaml:244-256`); gym and MuJoCo are absent here, so the
model is restated from humanoid.xml: 13 bodies under the world (torso on a free
joint; lwaist, pelvis, two thigh / shin / foot chains, two upper / lower arms), 17
hinges with their axes, anchors, ranges, stiffness, damping and armature, capsule /
sphere geoms (``inertiafromgeom``: density 1000), and 17 motors with their gears.

``compile_model()`` turns the tables into the per-body / per-dof arrays the dynamics
use (body mass, COM and inertia about the COM in the body frame; dof parents, axes,
anchors; contact spheres at the geoms' end caps).  ``write_header()`` emits the same
numbers as ``csrc/humanoid_model.h`` (17 significant digits, so the device constants
are the float64 values the numpy twin uses).

    python -m modular_rl_amd.humanoid_model      (rewrites csrc/humanoid_model.h)
"""
import math
import os

import numpy as np

DENSITY = 1000.0
DEG = math.pi / 180.0

# (name, parent, pos in parent, quat in parent [w x y z], geoms); geoms:
# ("capsule", from, to, radius) | ("sphere", center, radius), body frame
BODIES = [
    ("torso", -1, (0.0, 0.0, 1.4), (1.0, 0.0, 0.0, 0.0),
     [("capsule", (0.0, -0.07, 0.0), (0.0, 0.07, 0.0), 0.07), ("sphere", (0.0, 0.0, 0.19), 0.09),
      ("capsule", (-0.01, -0.06, -0.12), (-0.01, 0.06, -0.12), 0.06)]),
    ("lwaist", 0, (-0.01, 0.0, -0.26), (1.0, 0.0, -0.002, 0.0),
     [("capsule", (0.0, -0.06, 0.0), (0.0, 0.06, 0.0), 0.06)]),
    ("pelvis", 1, (0.0, 0.0, -0.165), (1.0, 0.0, -0.002, 0.0),
     [("capsule", (-0.02, -0.07, 0.0), (-0.02, 0.07, 0.0), 0.09)]),
    ("right_thigh", 2, (0.0, -0.1, -0.04), (1.0, 0.0, 0.0, 0.0),
     [("capsule", (0.0, 0.0, 0.0), (0.0, 0.01, -0.34), 0.06)]),
    ("right_shin", 3, (0.0, 0.01, -0.403), (1.0, 0.0, 0.0, 0.0),
     [("capsule", (0.0, 0.0, 0.0), (0.0, 0.0, -0.3), 0.049)]),
    ("right_foot", 4, (0.0, 0.0, -0.45), (1.0, 0.0, 0.0, 0.0),
     [("sphere", (0.0, 0.0, 0.1), 0.075)]),
    ("left_thigh", 2, (0.0, 0.1, -0.04), (1.0, 0.0, 0.0, 0.0),
     [("capsule", (0.0, 0.0, 0.0), (0.0, -0.01, -0.34), 0.06)]),
    ("left_shin", 6, (0.0, -0.01, -0.403), (1.0, 0.0, 0.0, 0.0),
     [("capsule", (0.0, 0.0, 0.0), (0.0, 0.0, -0.3), 0.049)]),
    ("left_foot", 7, (0.0, 0.0, -0.45), (1.0, 0.0, 0.0, 0.0),
     [("sphere", (0.0, 0.0, 0.1), 0.075)]),
    ("right_upper_arm", 0, (0.0, -0.17, 0.06), (1.0, 0.0, 0.0, 0.0),
     [("capsule", (0.0, 0.0, 0.0), (0.16, -0.16, -0.16), 0.04)]),
    ("right_lower_arm", 9, (0.18, -0.18, -0.18), (1.0, 0.0, 0.0, 0.0),
     [("capsule", (0.01, 0.01, 0.01), (0.17, 0.17, 0.17), 0.031), ("sphere", (0.18, 0.18, 0.18), 0.04)]),
    ("left_upper_arm", 0, (0.0, 0.17, 0.06), (1.0, 0.0, 0.0, 0.0),
     [("capsule", (0.0, 0.0, 0.0), (0.16, 0.16, -0.16), 0.04)]),
    ("left_lower_arm", 11, (0.18, 0.18, -0.18), (1.0, 0.0, 0.0, 0.0),
     [("capsule", (0.01, -0.01, 0.01), (0.17, -0.17, 0.17), 0.031), ("sphere", (0.18, -0.18, 0.18), 0.04)]),
]

# hinges in qpos order: (name, body, axis, anchor, range [deg], stiffness, damping, armature);
# humanoid.xml's <default> gives damping 1 where a joint names none
HINGES = [
    ("abdomen_z", 1, (0, 0, 1), (0, 0, 0.065), (-45, 45), 20.0, 5.0, 0.02),
    ("abdomen_y", 1, (0, 1, 0), (0, 0, 0.065), (-75, 30), 10.0, 5.0, 0.02),
    ("abdomen_x", 2, (1, 0, 0), (0, 0, 0.1), (-35, 35), 10.0, 5.0, 0.02),
    ("right_hip_x", 3, (1, 0, 0), (0, 0, 0), (-25, 5), 10.0, 5.0, 0.01),
    ("right_hip_z", 3, (0, 0, 1), (0, 0, 0), (-60, 35), 10.0, 5.0, 0.01),
    ("right_hip_y", 3, (0, 1, 0), (0, 0, 0), (-110, 20), 20.0, 5.0, 0.008),
    ("right_knee", 4, (0, -1, 0), (0, 0, 0.02), (-160, -2), 0.0, 1.0, 0.006),
    ("left_hip_x", 6, (-1, 0, 0), (0, 0, 0), (-25, 5), 10.0, 5.0, 0.01),
    ("left_hip_z", 6, (0, 0, -1), (0, 0, 0), (-60, 35), 10.0, 5.0, 0.01),
    ("left_hip_y", 6, (0, 1, 0), (0, 0, 0), (-110, 20), 20.0, 5.0, 0.01),
    ("left_knee", 7, (0, -1, 0), (0, 0, 0.02), (-160, -2), 1.0, 1.0, 0.006),
    ("right_shoulder1", 9, (2, 1, 1), (0, 0, 0), (-85, 60), 1.0, 1.0, 0.0068),
    ("right_shoulder2", 9, (0, -1, 1), (0, 0, 0), (-85, 60), 1.0, 1.0, 0.0051),
    ("right_elbow", 10, (0, -1, 1), (0, 0, 0), (-90, 50), 0.0, 1.0, 0.0028),
    ("left_shoulder1", 11, (2, -1, 1), (0, 0, 0), (-60, 85), 1.0, 1.0, 0.0068),
    ("left_shoulder2", 11, (0, 1, 1), (0, 0, 0), (-60, 85), 1.0, 1.0, 0.0051),
    ("left_elbow", 12, (0, -1, -1), (0, 0, 0), (-90, 50), 0.0, 1.0, 0.0028),
]

# motors in ctrl order (humanoid.xml <actuator>): (joint, gear); ctrlrange -0.4 .. 0.4
MOTORS = [("abdomen_y", 100), ("abdomen_z", 100), ("abdomen_x", 100), ("right_hip_x", 100), ("right_hip_z", 100),
          ("right_hip_y", 300), ("right_knee", 200), ("left_hip_x", 100), ("left_hip_z", 100), ("left_hip_y", 300),
          ("left_knee", 200), ("right_shoulder1", 25), ("right_shoulder2", 25), ("right_elbow", 25),
          ("left_shoulder1", 25), ("left_shoulder2", 25), ("left_elbow", 25)]
CTRL_LIMIT = 0.4

NB = len(BODIES)          # 13 bodies (MuJoCo body ids 1..13; id 0 is the world)
NQ, NV, NACT = 24, 23, 17


def _capsule(a, b, r):
    """mass, COM and inertia about the COM (3x3) of a capsule of uniform density:
    a cylinder of the segment's length and two hemispherical caps."""
    a, b = np.asarray(a, float), np.asarray(b, float)
    d = b - a
    h = float(np.linalg.norm(d))
    u = d / h
    m_cyl = DENSITY * math.pi * r * r * h
    m_sph = DENSITY * 4.0 / 3.0 * math.pi * r ** 3
    m = m_cyl + m_sph
    i_ax = m_cyl * r * r / 2.0 + m_sph * 2.0 * r * r / 5.0
    # each hemisphere: 83/320 m_hemi r^2 about its own COM, COM 3r/8 beyond the segment end
    m_h = m_sph / 2.0
    i_h = 83.0 / 320.0 * m_h * r * r
    dz = h / 2.0 + 3.0 * r / 8.0
    i_perp = m_cyl * (r * r / 4.0 + h * h / 12.0) + 2.0 * (i_h + m_h * dz * dz)
    inertia = i_perp * (np.eye(3) - np.outer(u, u)) + i_ax * np.outer(u, u)
    return m, (a + b) / 2.0, inertia


def _sphere(c, r):
    m = DENSITY * 4.0 / 3.0 * math.pi * r ** 3
    return m, np.asarray(c, float), 2.0 / 5.0 * m * r * r * np.eye(3)


def compile_model():
    """Arrays of the model (float64 / int):
    body_parent[NB] (-1 = world), body_pos[NB, 3], body_quat[NB, 4], body_mass[NB],
    body_ipos[NB, 3], body_inertia[NB, 6] (xx yy zz xy xz yz about the COM, body frame),
    hinge_* [17], dof_parent[NV], dof_body[NV], act_dof[17], act_gear[17],
    sphere_body / sphere_pos / sphere_r (contact spheres: capsule end caps, spheres)."""
    M = {}
    M["body_parent"] = np.array([b[1] for b in BODIES], dtype=np.int64)
    M["body_pos"] = np.array([b[2] for b in BODIES], dtype=np.float64)
    q = np.array([b[3] for b in BODIES], dtype=np.float64)
    M["body_quat"] = q / np.linalg.norm(q, axis=1, keepdims=True)
    mass, ipos, inert = [], [], []
    sb, sp, sr = [], [], []
    for bi, (_, _, _, _, geoms) in enumerate(BODIES):
        parts = []
        for g in geoms:
            if g[0] == "capsule":
                parts.append(_capsule(g[1], g[2], g[3]))
                for end in (g[1], g[2]):
                    sb.append(bi)
                    sp.append(end)
                    sr.append(g[3])
            else:
                parts.append(_sphere(g[1], g[2]))
                sb.append(bi)
                sp.append(g[1])
                sr.append(g[2])
        m = sum(p[0] for p in parts)
        c = sum(p[0] * p[1] for p in parts) / m
        inertia = np.zeros((3, 3))
        for pm, pc, pi in parts:
            d = pc - c
            inertia += pi + pm * (np.dot(d, d) * np.eye(3) - np.outer(d, d))
        mass.append(m)
        ipos.append(c)
        inert.append([inertia[0, 0], inertia[1, 1], inertia[2, 2], inertia[0, 1], inertia[0, 2], inertia[1, 2]])
    M["body_mass"] = np.array(mass)
    M["body_ipos"] = np.array(ipos)
    M["body_inertia"] = np.array(inert)
    M["sphere_body"] = np.array(sb, dtype=np.int64)
    M["sphere_pos"] = np.array(sp, dtype=np.float64)
    M["sphere_r"] = np.array(sr, dtype=np.float64)
    ax = np.array([h[2] for h in HINGES], dtype=np.float64)
    M["hinge_body"] = np.array([h[1] for h in HINGES], dtype=np.int64)
    M["hinge_axis"] = ax / np.linalg.norm(ax, axis=1, keepdims=True)
    M["hinge_pos"] = np.array([h[3] for h in HINGES], dtype=np.float64)
    M["hinge_lo"] = np.array([h[4][0] * DEG for h in HINGES])
    M["hinge_hi"] = np.array([h[4][1] * DEG for h in HINGES])
    M["hinge_stiff"] = np.array([h[5] for h in HINGES])
    M["hinge_damp"] = np.array([h[6] for h in HINGES])
    M["hinge_arm"] = np.array([h[7] for h in HINGES])
    # dofs: 0-2 root translation, 3-5 root rotation (local axes), 6.. hinges in order;
    # a dof's parent is the previous dof of its body, else the last dof of the parent body
    dof_body = [0] * 6 + [h[1] for h in HINGES]
    last = {0: 5}
    dof_parent = [-1, 0, 1, 2, 3, 4]
    for j, h in enumerate(HINGES):
        b = h[1]
        d = 6 + j
        if b in last:
            dof_parent.append(last[b])
        else:
            p = BODIES[b][1]
            while p not in last:
                p = BODIES[p][1]
            dof_parent.append(last[p])
        last[b] = d
    M["dof_body"] = np.array(dof_body, dtype=np.int64)
    M["dof_parent"] = np.array(dof_parent, dtype=np.int64)
    names = [h[0] for h in HINGES]
    M["act_dof"] = np.array([6 + names.index(j) for j, _ in MOTORS], dtype=np.int64)
    M["act_gear"] = np.array([g for _, g in MOTORS], dtype=np.float64)
    # first hinge of each body and its count (bodies 1..12 carry 1-3 hinges)
    first, count = [], []
    for b in range(NB):
        idx = [j for j, h in enumerate(HINGES) if h[1] == b]
        first.append(idx[0] if idx else 0)
        count.append(len(idx))
    M["body_hinge0"] = np.array(first, dtype=np.int64)
    M["body_nhinge"] = np.array(count, dtype=np.int64)
    # tree levels (root 0), bodies by level; each body's children (descending index,
    # the order a leaves-first sweep adds them); each body's contact spheres
    depth = [0] * NB
    for b in range(1, NB):
        depth[b] = depth[BODIES[b][1]] + 1
    levels = [[b for b in range(NB) if depth[b] == d] for d in range(max(depth) + 1)]
    M["level_start"] = np.cumsum([0] + [len(lv) for lv in levels]).astype(np.int64)
    M["level_bodies"] = np.array([b for lv in levels for b in lv], dtype=np.int64)
    kids = [[c for c in range(NB - 1, 0, -1) if BODIES[c][1] == b] for b in range(NB)]
    M["child_start"] = np.cumsum([0] + [len(k) for k in kids]).astype(np.int64)
    M["children"] = np.array([c for k in kids for c in k] + [0], dtype=np.int64)
    sph0 = [int(np.argmax(np.array(sb) == b)) if b in sb else 0 for b in range(NB)]
    M["body_sph0"] = np.array(sph0, dtype=np.int64)
    M["body_nsph"] = np.array([sb.count(b) for b in range(NB)], dtype=np.int64)
    # dof-tree tables of the L^T D L factorisation (leaves first) and of the solves
    dpar = M["dof_parent"]

    def chain(i):  # i and its ancestors, nearest first
        out = []
        while i >= 0:
            out.append(int(i))
            i = dpar[i]
        return out
    pi, pj, pstart = [], [], [0]
    for k in range(NV):
        for i in chain(k)[1:]:
            for j in chain(i):
                pi.append(i)
                pj.append(j)
        pstart.append(len(pi))
    M["ldl_start"] = np.array(pstart, dtype=np.int64)
    M["ldl_i"] = np.array(pi, dtype=np.int64)
    M["ldl_j"] = np.array(pj, dtype=np.int64)
    desc, dstart = [], [0]
    for j in range(NV):
        desc += [i for i in range(j + 1, NV) if j in chain(i)]
        dstart.append(len(desc))
    M["desc_start"] = np.array(dstart, dtype=np.int64)
    M["desc"] = np.array(desc, dtype=np.int64)
    # a-th strict ancestor of each dof (-1 past the root): ANC[k][a]
    anc = -np.ones((NV, 16), dtype=np.int64)
    for k in range(NV):
        ch = chain(k)[1:]
        anc[k, :len(ch)] = ch
    M["anc"] = anc
    return M


MODEL = compile_model()


def _fmt(v):
    return repr(float(v))


def write_header(path=None):
    path = path or os.path.join(os.path.dirname(os.path.abspath(__file__)), "csrc", "humanoid_model.h")
    M = MODEL

    def arr(name, a, ctype="double"):
        a = np.asarray(a).ravel()
        vals = ", ".join(_fmt(x) if ctype == "double" else str(int(x)) for x in a)
        return f"constexpr {ctype} {name}[{a.size}] = {{{vals}}};\n"

    out = ["// GENERATED by `python -m modular_rl_amd.humanoid_model` from humanoid_model.py\n",
           "// (gym humanoid.xml tables + compiled mass properties).  Do not edit.\n",
           "#pragma once\n\nnamespace mrl {\nnamespace hm {\n\n",
           f"constexpr int NB = {NB}, NQ = {NQ}, NV = {NV}, NACT = {NACT}, NSPH = {len(M['sphere_r'])};\n"]
    out.append(arr("BODY_PARENT", M["body_parent"], "int"))
    out.append(arr("BODY_POS", M["body_pos"]))
    out.append(arr("BODY_QUAT", M["body_quat"]))
    out.append(arr("BODY_MASS", M["body_mass"]))
    out.append(arr("BODY_IPOS", M["body_ipos"]))
    out.append(arr("BODY_INERTIA", M["body_inertia"]))
    out.append(arr("BODY_HINGE0", M["body_hinge0"], "int"))
    out.append(arr("BODY_NHINGE", M["body_nhinge"], "int"))
    out.append(arr("SPHERE_BODY", M["sphere_body"], "int"))
    out.append(arr("SPHERE_POS", M["sphere_pos"]))
    out.append(arr("SPHERE_R", M["sphere_r"]))
    out.append(arr("HINGE_AXIS", M["hinge_axis"]))
    out.append(arr("HINGE_POS", M["hinge_pos"]))
    out.append(arr("HINGE_LO", M["hinge_lo"]))
    out.append(arr("HINGE_HI", M["hinge_hi"]))
    out.append(arr("HINGE_STIFF", M["hinge_stiff"]))
    out.append(arr("HINGE_DAMP", M["hinge_damp"]))
    out.append(arr("HINGE_ARM", M["hinge_arm"]))
    out.append(arr("DOF_BODY", M["dof_body"], "int"))
    out.append(arr("DOF_PARENT", M["dof_parent"], "int"))
    out.append(arr("ACT_DOF", M["act_dof"], "int"))
    out.append(arr("ACT_GEAR", M["act_gear"]))
    out.append(f"constexpr int NLEVEL = {len(M['level_start']) - 1};\n")
    for name in ("level_start", "level_bodies", "child_start", "children", "body_sph0", "body_nsph", "ldl_start",
                 "ldl_i", "ldl_j", "desc_start", "desc", "anc"):
        out.append(arr(name.upper(), M[name], "int"))
    out.append(f"constexpr double TOTAL_MASS = {_fmt(M['body_mass'].sum())};\n")
    out.append("\n}  // namespace hm\n}  // namespace mrl\n")
    with open(path, "w") as f:
        f.write("".join(out))
    return path


if __name__ == "__main__":
    print(write_header())
