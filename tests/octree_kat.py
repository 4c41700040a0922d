"""Known-answer case for the reference's octree traversal, derived by hand from
`Octree::_intersect_recurse` (geometry.rs:1245-1295) and `Octree::_build` (:1149-1216), independent
of the oracle's restatement.

Mesh (14 triangles, bbox exactly [0,4]^3 from its vertices, geometry.rs:777-833):
  tri 0  T_near  x = 1.3, corners (y,z) = (0.2,0.2) (0.9,0.2) (0.2,0.9)
  tri 1  T_far   x = 0.5, same corners
  tri 2  anchor  (0,0,0) (0.1,0,0) (0,0.1,0)          -> bbox min
  tri 3  anchor  (4,4,4) (3.9,4,4) (4,3.9,4)          -> bbox max
  tri 4-8   fillers in [1.05,1.45]^3 (x = 1.10 .. 1.30)
  tri 9-13  fillers in [1.55,1.95]^3 (x = 1.60 .. 1.80)

Build (SMALL_NODE = 9, MAX_DEPTH = 10; a triangle goes to every octant it overlaps):
  root [0,4]^3: 14 > 9 -> parent. Octant 0 = [0,2]^3 gets tris 0,1,2,4-13 (13), octant 7 = [2,4]^3
  gets tri 3 (leaf). Node [0,2]^3: 13 > 9 -> parent; its octant 0 = [0,1]^3 gets tris 1,2 (leaf),
  octant 4 = [1,2]x[0,1]x[0,1] gets tri 0 (leaf), octant 7 = [1,2]^3 gets the 10 fillers -> parent
  with two leaves of 5 ([1,1.5]^3 and [1.5,2]^3). 8 nodes: 3 parents, 5 leaves, 14 triangle refs (1 + 2 + 1 + 5 + 5).

Ray: o = (1.7, 0.5, 0.5), d = (-1, 0.01, 0.02) / |(-1, 0.01, 0.02)|. Along the ray it meets T_near
first (x = 1.3, t = 0.4 / |d_x| ~ 0.4001) and T_far later (x = 0.5, t = 1.2 / |d_x| ~ 1.2003).
Traversal: the child order is fixed per ray by the distances from o to the ROOT octant centres
(geometry.rs:1248-1260): octant 0 (centre (1,1,1), 0.995), 4 ((3,1,1), 1.480), 1 and 2 (2.641, a tie
kept in index order), 5 and 6 (2.858), 3 (3.604), 7 (3.766): order 0,4,1,2,5,6,3,7 — reused at every
level. At the root, octant 0's box is hit (o is inside it: its -x face at t ~ 1.7) -> recurse into
node [0,2]^3. There the same order visits ITS octant 0 = [0,1]^3 first; the ray hits that box (its
-x face x = 0 at t ~ 1.7004, point (0, 0.517, 0.534) inside the face) -> recurse into the leaf
{T_far, anchor}: T_far is hit (t ~ 1.2003) and returned (geometry.rs:1267-1269: the first subtree
with any hit wins). T_near, in octant 4 of that node, is never visited.

Expected: Octree::intersect returns T_far's hit, t = 1.2 / |d_x| (the farther triangle); the
nearest-triangle semantics (`octree: None`, geometry.rs:886-903) return T_near at t = 0.4 / |d_x|.
Control ray (o = (0.3, 0.5, 0.5), d ~ +x): both semantics return T_far at t = 0.2 / |d_x|.
"""
import numpy as np

T_NEAR_X, T_FAR_X = 1.3, 0.5


def _yz_tri(x, lo, hi):
    return [(x, lo, lo), (x, hi, lo), (x, lo, hi)]


def obj_text():
    tris = [_yz_tri(T_NEAR_X, 0.2, 0.9), _yz_tri(T_FAR_X, 0.2, 0.9),
            [(0, 0, 0), (0.1, 0, 0), (0, 0.1, 0)], [(4, 4, 4), (3.9, 4, 4), (4, 3.9, 4)]]
    tris += [_yz_tri(1.10 + 0.05 * k, 1.1, 1.4) for k in range(5)]
    tris += [_yz_tri(1.60 + 0.05 * k, 1.6, 1.9) for k in range(5)]
    lines, n = [], 0
    for t in tris:
        for v in t:
            lines.append("v %r %r %r" % tuple(float(c) for c in v))
        lines.append("f %d %d %d" % (n + 1, n + 2, n + 3))
        n += 3
    return "\n".join(lines) + "\n"


SCENE = """
[camera]
pos = [2.0, 2.0, 40.0]
dir = [0.0, 0.0, -1.0]
[[objects]]
brdf = { type = "diffuse", kd = [0.75, 0.75, 0.75] }
geometry = { type = "mesh", path = "kat.obj" }
[[objects]]
emitted = [50.0, 50.0, 50.0]
brdf = { type = "diffuse", kd = [0.0, 0.0, 0.0] }
geometry = { type = "sphere", pos = [50.0, 70.0, 100.0], r = 4.0 }
"""


def write_scene(tmp_path):
    (tmp_path / "assets").mkdir(exist_ok=True)
    (tmp_path / "assets" / "kat.obj").write_text(obj_text())
    p = tmp_path / "kat.toml"
    p.write_text(SCENE)
    return str(p)


def rays():
    d = np.array([[-1.0, 0.01, 0.02], [1.0, 0.01, 0.02]])
    d /= np.linalg.norm(d, axis=1, keepdims=True)
    o = np.array([[1.7, 0.5, 0.5], [0.3, 0.5, 0.5]])
    return o, d


def expected_t(d):
    """(octree semantics, nearest semantics) hit distances of the two rays, from the plane x = X:
    t = (X - o_x) / d_x."""
    dx = d[:, 0]
    return np.array([(T_FAR_X - 1.7) / dx[0], (T_FAR_X - 0.3) / dx[1]]), \
        np.array([(T_NEAR_X - 1.7) / dx[0], (T_FAR_X - 0.3) / dx[1]])
