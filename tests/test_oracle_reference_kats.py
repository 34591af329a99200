"""Pin the oracle with the reference's own unit tests.

Each test restates one #[test] of the Rust reference against the C oracle:
  test_camera              src/camera/mod.rs:315-343
  test_rotate_matrix       src/algebra/transform.rs:637-663 (asserted part)
  test_matrix_multiplication  src/algebra/transform.rs:665-691
  test_bound_transform     src/world/shapes/mod.rs:880-899
plus rand 0.8's documented float conversions (the RNG boundary, §8a-19).
"""
import ctypes as C
import math

import numpy as np

import oracle as O


def approx_equal(a, b):  # src/algebra/mod.rs:14-17
    return abs(a - b) < 1e-15


def d(v):
    return (C.c_double * len(v))(*v)


def test_camera():
    L = O.lib()
    cam = O.Camera()
    L.or_camera_new(d([0, 0, 0]), d([0, 0, -1]), d([0, 1, 0]), 1.0, L.or_to_radians(90.0), C.byref(cam))
    assert all(approx_equal(a, b) for a, b in zip(cam.right, [1.0, 0.0, 0.0]))
    k = O.Caster()
    L.or_caster_new(C.byref(cam), 1920, 1080, C.byref(k))
    assert approx_equal(k.pixel_resolution, 2.0 / 1920)
    # ray_caster.len() == w*h: the oracle renders exactly the listed pixels
    assert k.width * k.height == 1920 * 1080


def test_rotate_matrix():
    L = O.lib()
    m = (C.c_double * 16)()
    L.or_rotate(d([0.0, -90.0, 0.0]), m)
    M = np.array(m[:]).reshape(4, 4)
    v = np.array([0.0, 0.0, -1.0, 1.0])
    # Mul<Vector3d> for Transform: x = v.x*m00 + v.y*m01 + v.z*m02 + m03 (transform.rs:505-515)
    v1 = [v[0] * M[i, 0] + v[1] * M[i, 1] + v[2] * M[i, 2] + M[i, 3] for i in range(3)]
    assert approx_equal(v1[0], 1.0) and approx_equal(v1[1], 0.0) and approx_equal(v1[2], 0.0)


def test_matrix_multiplication():
    L = O.lib()
    m1 = d([float(x) for x in range(1, 17)])
    m2 = d([float(x) for x in range(17, 33)])
    out = (C.c_double * 16)()
    L.or_mat_mul(m1, m2, out)
    M = np.array(out[:]).reshape(4, 4)
    assert M[0, 0] == 250.0 and M[1, 0] == 618.0 and M[2, 3] == 1112.0
    L.or_mat_mul(m2, m1, out)
    M = np.array(out[:]).reshape(4, 4)
    assert M[0, 0] == 538.0 and M[1, 0] == 650.0 and M[2, 3] == 1080.0


def test_bound_transform():
    L = O.lib()
    direct, inverse = (C.c_double * 16)(), (C.c_double * 16)()
    L.or_transform_new(d([-10.0, 5.0, 2.5]), d([0, 0, 0]), d([2.0, 2.0, 2.0]), direct, inverse)
    mn, mx = (C.c_double * 3)(), (C.c_double * 3)()
    L.or_aabb_transform(d([-1, -1, -1]), d([1, 1, 1]), direct, mn, mx)
    for got, want in zip(list(mn) + list(mx), [-12.0, 3.0, 0.5, -8.0, 7.0, 4.5]):
        assert approx_equal(want, got)


def test_inverse_transform_is_inverse():
    """InversableTransform::new builds inverse = S^-1 R^-1 T^-1 (transform.rs:16-23)."""
    L = O.lib()
    direct, inverse = (C.c_double * 16)(), (C.c_double * 16)()
    L.or_transform_new(d([212.5, 200, 147.5]), d([-95.0, -18.0, 0.0]), d([82.5, 82.5, 82.5]), direct, inverse)
    P = np.array(direct[:]).reshape(4, 4) @ np.array(inverse[:]).reshape(4, 4)
    assert np.allclose(P, np.eye(4), atol=1e-12)


def test_to_radians():
    # f64::to_radians = self * (PI / 180.0)
    assert O.lib().or_to_radians(40.0) == 40.0 * (math.pi / 180.0)


def test_rand_float_conversions():
    """rand 0.8: Standard f64 = (u >> 11) * 2^-53; UniformFloat::new_inclusive(-1, 1)
    has scale = 2 + 2^-51 after its inclusive-bound loop; (0, 1) has 1 + 2^-52."""
    L = O.lib()
    assert L.or_uniform_incl_scale(-1.0, 1.0) == 2.0 + 2.0 ** -51
    assert L.or_uniform_incl_scale(0.0, 1.0) == 1.0 + 2.0 ** -52
    st = C.c_uint64(12345)
    s2 = C.c_uint64(12345)
    u = L.or_rng_next(C.byref(s2))
    assert L.or_gen_f64(C.byref(st)) == (u >> 11) * 2.0 ** -53
    # the largest draw stays inside the inclusive range
    scale = L.or_uniform_incl_scale(-1.0, 1.0)
    top = (2.0 - 2.0 ** -52) - 1.0
    assert top * scale + -1.0 <= 1.0


def test_splitmix_reference_vector():
    """SplitMix64 finaliser (Steele et al. 2014): first outputs from state 0 are the
    published constants of the algorithm."""
    L = O.lib()
    st = C.c_uint64(0)
    outs = [L.or_rng_next(C.byref(st)) for _ in range(3)]
    assert outs == [0xE220A8397B1DCDAF, 0x6E789E6AA1B965F4, 0x06C45D188009454F]
