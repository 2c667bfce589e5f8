"""Writes the golden fixtures under tests/golden/ (run: python tests/golden/make_golden.py).

Every vector below is a literal input/expected-output pair transcribed from the
reference's own tests (paths relative to the reference root).  The reference
cannot be built or imported here (TensorFlow 1.15 fork,
Bazel 0.24.1, network-fetched deps, TF not installed), so these KATs are what
pins the CPU restatement in oracle/.  Formula-defined KATs (the 262144-row
segment tests) are stored as their generating parameters plus expectation
formulas evaluated here in float32 exactly as the reference test does.
"""
import json
import os

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))


def f32(xs):
    return [float(np.float32(x)) for x in xs]


def fused_local():
    # core/kernels/fused_embedding/fused_embedding_local_ops_test.cc
    table = list(range(128))                                   # :161-176 (16 x 8, 0..127)
    sp_values = [3, 1, 4, 5, 7, 3, 12, 12, 15, 4]             # :154
    sp_indices = [0, 1, 0, 5, 1, 2, 1, 1, 1, 7,                # :155-156
                  2, 1, 2, 4, 2, 7, 3, 0, 3, 6]
    fwd = {
        "sqrtn": dict(max_norm=-1.0, expected=[                # :63-75
            22.627416610717773, 24.0416316986084, 25.45584487915039,
            26.870058059692383, 28.284271240234375, 29.698484420776367,
            31.112699508666992, 32.526912689208984, 73.90083312988281,
            75.63288879394531, 77.36493682861328, 79.09698486328125,
            80.82904052734375, 82.56108856201172, 84.29314422607422,
            86.02519226074219, 124.70765686035156, 126.43971252441406,
            128.17176818847656, 129.90380859375, 131.6358642578125,
            133.367919921875, 135.09996032714844, 136.83201599121094,
            107.48023223876953, 108.89444732666016, 110.30866241455078,
            111.72286987304688, 113.1370849609375, 114.55130004882812,
            115.96551513671875, 117.37973022460938]),
        "mean": dict(max_norm=-1.0, expected=[                 # :78-90
            16, 17, 18, 19, 20, 21, 22, 23, 42.66666793823242,
            43.66666793823242, 44.66666793823242, 45.66666793823242,
            46.66666793823242, 47.66666793823242, 48.66666793823242,
            49.66666793823242, 72, 73, 74, 75, 76, 77, 78, 79,
            76, 77, 78, 79, 80, 81, 82, 83]),
        "sum": dict(max_norm=-1.0, expected=[                  # :93-99
            32, 34, 36, 38, 40, 42, 44, 46, 128, 131, 134, 137, 140, 143, 146, 149,
            216, 219, 222, 225, 228, 231, 234, 237, 152, 154, 156, 158, 160, 162, 164, 166]),
        "sqrtn_maxnorm200": dict(combiner="sqrtn", max_norm=200.0, expected=[  # :102-111
            22.62741661, 24.04163170, 25.45584488, 26.87005806, 28.28427124,
            29.69848442, 31.11269951, 32.52691269, 73.90083313, 75.63288879,
            77.36493683, 79.09698486, 80.82904053, 82.56108856, 84.29314423,
            86.02519226, 92.61308289, 94.01081848, 95.40855408, 96.80628204,
            98.20401764, 99.60175323, 100.99948120, 102.39721680, 71.20205688,
            72.31395721, 73.42584991, 74.53774261, 75.64963531, 76.76153564,
            77.87342834, 78.98532867]),
    }
    top_grad = list(range(32))                                  # :330-333
    grad = {
        "sqrtn": dict(max_norm=-1.0, expected=[                # :207-233
            0.0, 0.7071067690849304, 1.4142135381698608, 2.1213204860687256,
            2.8284270763397217, 3.535533905029297, 4.242640972137451, 4.949747562408447,
            0.0, 0.7071067690849304, 1.4142135381698608, 2.1213204860687256,
            2.8284270763397217, 3.535533905029297, 4.242640972137451, 4.949747562408447,
            4.618802070617676, 5.196152687072754, 5.773502826690674, 6.350852966308594,
            6.928203582763672, 7.505553722381592, 8.082903861999512, 8.66025447845459,
            4.618802070617676, 5.196152687072754, 5.773502826690674, 6.350852966308594,
            6.928203582763672, 7.505553722381592, 8.082903861999512, 8.66025447845459,
            4.618802070617676, 5.196152687072754, 5.773502826690674, 6.350852966308594,
            6.928203582763672, 7.505553722381592, 8.082903861999512, 8.66025447845459,
            9.237604141235352, 9.81495475769043, 10.392305374145508, 10.96965503692627,
            11.547005653381348, 12.124356269836426, 12.701705932617188, 13.279056549072266,
            9.237604141235352, 9.81495475769043, 10.392305374145508, 10.96965503692627,
            11.547005653381348, 12.124356269836426, 12.701705932617188, 13.279056549072266,
            9.237604141235352, 9.81495475769043, 10.392305374145508, 10.96965503692627,
            11.547005653381348, 12.124356269836426, 12.701705932617188, 13.279056549072266,
            16.970563888549805, 17.677669525146484, 18.384777069091797, 19.091882705688477,
            19.79899024963379, 20.5060977935791, 21.21320343017578, 21.920310974121094,
            16.970563888549805, 17.677669525146484, 18.384777069091797, 19.091882705688477,
            19.79899024963379, 20.5060977935791, 21.21320343017578, 21.920310974121094]),
        "mean": dict(max_norm=-1.0, expected=[                 # :236-262
            0.0, 0.5, 1.0, 1.5, 2.0, 2.5, 3.0, 3.5,
            0.0, 0.5, 1.0, 1.5, 2.0, 2.5, 3.0, 3.5,
            2.6666667461395264, 3.0, 3.3333332538604736, 3.6666667461395264, 4.0,
            4.333333492279053, 4.666666507720947, 5.0,
            2.6666667461395264, 3.0, 3.3333332538604736, 3.6666667461395264, 4.0,
            4.333333492279053, 4.666666507720947, 5.0,
            2.6666667461395264, 3.0, 3.3333332538604736, 3.6666667461395264, 4.0,
            4.333333492279053, 4.666666507720947, 5.0,
            5.333333492279053, 5.666666507720947, 6.0, 6.333333492279053, 6.666666507720947,
            7.0, 7.333333492279053, 7.666666507720947,
            5.333333492279053, 5.666666507720947, 6.0, 6.333333492279053, 6.666666507720947,
            7.0, 7.333333492279053, 7.666666507720947,
            5.333333492279053, 5.666666507720947, 6.0, 6.333333492279053, 6.666666507720947,
            7.0, 7.333333492279053, 7.666666507720947,
            12.0, 12.5, 13.0, 13.5, 14.0, 14.5, 15.0, 15.5,
            12.0, 12.5, 13.0, 13.5, 14.0, 14.5, 15.0, 15.5]),
        "sum": dict(max_norm=-1.0, expected=[                  # :265-273
            0, 1, 2, 3, 4, 5, 6, 7, 0, 1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11, 12, 13, 14, 15,
            8, 9, 10, 11, 12, 13, 14, 15, 8, 9, 10, 11, 12, 13, 14, 15,
            16, 17, 18, 19, 20, 21, 22, 23, 16, 17, 18, 19, 20, 21, 22, 23,
            16, 17, 18, 19, 20, 21, 22, 23, 24, 25, 26, 27, 28, 29, 30, 31,
            24, 25, 26, 27, 28, 29, 30, 31]),
        "mean_maxnorm100": dict(combiner="mean", max_norm=100.0, expected=[  # :276-288
            0.00000000, 0.50000000, 1.00000000, 1.50000000, 2.00000000, 2.50000000, 3.00000000, 3.50000000,
            0.00000000, 0.50000000, 1.00000000, 1.50000000, 2.00000000, 2.50000000, 3.00000000, 3.50000000,
            2.65028572, 2.98157120, 3.31285667, 3.64414287, 3.97542834, 4.30671406, 4.63799953, 4.96928549,
            2.16437674, 2.43492365, 2.70547056, 2.97601795, 3.24656487, 3.51711202, 3.78765893, 4.05820608,
            1.58337951, 1.78130186, 1.97922409, 2.17714667, 2.37506914, 2.57299161, 2.77091384, 2.96883631,
            5.33333349, 5.66666651, 6.00000000, 6.33333349, 6.66666651, 7.00000000, 7.33333349, 7.66666651,
            1.89459133, 2.01300311, 2.13141513, 2.24982715, 2.36823893, 2.48665094, 2.60506320, 2.72347474,
            1.89459133, 2.01300311, 2.13141513, 2.24982715, 2.36823893, 2.48665094, 2.60506320, 2.72347474,
            3.43474555, 3.57786012, 3.72097445, 3.86408877, 4.00720310, 4.15031767, 4.29343224, 4.43654633,
            11.92628479, 12.42321396, 12.92014217, 13.41707039, 13.91399956, 14.41092777, 14.90785599, 15.40478516]),
    }
    return dict(source="core/kernels/fused_embedding/fused_embedding_local_ops_test.cc",
                tolerance=1e-4, batch=4, dim=8, bucket=16, table=table,
                sp_values=sp_values, sp_indices=sp_indices, offsets_expected=[0, 2, 5, 8],
                forward=fwd, top_grad=top_grad, grad=grad)


def pre_lookup_partition():
    # core/kernels/fused_embedding/fused_embedding_ops_test.cc:59-97
    return dict(source="core/kernels/fused_embedding/fused_embedding_ops_test.cc:59-97",
                partition_rows=[6, 3, 7],
                sp_values=[1, 5, 3, 6, 12, 14, 15, 0, 5, 5, 11, 7],
                sp_indices=[2, 3, 4, 6, 1, 6, 12, 12, 12, 12, 11, 5,
                            15, 0, 11, 6, 7, 9, 11, 8, 12, 13, 13, 0],
                expected=[
                    dict(values=[0, 1, 3, 5, 5, 5], indices=[11, 6, 2, 3, 1, 6, 4, 6, 7, 9, 11, 8]),
                    dict(values=[0, 1], indices=[12, 12, 13, 0]),
                    dict(values=[2, 3, 5, 6], indices=[12, 13, 12, 12, 11, 5, 15, 0]),
                ])


def post_lookup():
    # core/kernels/fused_embedding/fused_embedding_ops_test.cc:129-196
    # (FusedEmbeddingSparsePostLookUp, 3 partitions, sqrtn, max_norm 200, tol 1e-4)
    # and :217-290 (PostLookUpGrad, 2 partitions, mean, max_norm 100, tol 1e-4)
    s0 = [8.0, 9.0, 10.0, 11.0, 12.0, 13.0, 14.0, 15.0, 24.0, 25.0,
          26.0, 27.0, 28.0, 29.0, 30.0, 31.0, 24.0, 25.0, 26.0, 27.0,
          28.0, 29.0, 30.0, 31.0, 32.0, 33.0, 34.0, 35.0, 36.0, 37.0,
          38.0, 39.0, 32.0, 33.0, 34.0, 35.0, 36.0, 37.0, 38.0, 39.0,
          40.0, 41.0, 42.0, 43.0, 44.0, 45.0, 46.0, 47.0]
    fwd = dict(source="core/kernels/fused_embedding/fused_embedding_ops_test.cc:129-196",
               combiner="sqrtn", max_norm=200.0, batch=4, cols=8, dim=8,
               shards=[s0, [56.0, 57.0, 58.0, 59.0, 60.0, 61.0, 62.0, 63.0],
                       [96.0, 97.0, 98.0, 99.0, 100.0, 101.0, 102.0, 103.0,
                        96.0, 97.0, 98.0, 99.0, 100.0, 101.0, 102.0, 103.0,
                        120.0, 121.0, 122.0, 123.0, 124.0, 125.0, 126.0, 127.0]],
               indices=[[0, 5, 0, 1, 2, 1, 1, 2, 3, 6, 1, 1], [1, 7], [2, 4, 2, 7, 3, 0]],
               expected=[22.62741661, 24.04163170, 25.45584488, 26.87005806, 28.28427124,
                         29.69848442, 31.11269951, 32.52691269, 73.90083313, 75.63288879,
                         77.36493683, 79.09698486, 80.82904053, 82.56108856, 84.29314423,
                         86.02519226, 92.61308289, 94.01081848, 95.40855408, 96.80628204,
                         98.20401764, 99.60175323, 100.99948120, 102.39721680, 71.20205688,
                         72.31395721, 73.42584991, 74.53774261, 75.64963531, 76.76153564,
                         77.87342834, 78.98532867],
               feature_nums=[2, 3, 3, 2], tol=1e-4)
    grad = dict(source="core/kernels/fused_embedding/fused_embedding_ops_test.cc:217-290",
                combiner="mean", max_norm=100.0, batch=4, dim=8,
                top_grad=[float(x) for x in range(32)],
                shards=[s0, [56.0, 57.0, 58.0, 59.0, 60.0, 61.0, 62.0, 63.0,
                             96.0, 97.0, 98.0, 99.0, 100.0, 101.0, 102.0, 103.0,
                             96.0, 97.0, 98.0, 99.0, 100.0, 101.0, 102.0, 103.0,
                             120.0, 121.0, 122.0, 123.0, 124.0, 125.0, 126.0, 127.0]],
                indices=[[0, 5, 0, 1, 2, 1, 1, 2, 3, 6, 1, 1], [1, 7, 2, 4, 2, 7, 3, 0]],
                feature_nums=[2, 3, 3, 2],
                expected=[[0.00000000, 0.50000000, 1.00000000, 1.50000000, 2.00000000,
                           2.50000000, 3.00000000, 3.50000000, 0.00000000, 0.50000000,
                           1.00000000, 1.50000000, 2.00000000, 2.50000000, 3.00000000,
                           3.50000000, 5.33333349, 5.66666651, 6.00000000, 6.33333349,
                           6.66666651, 7.00000000, 7.33333349, 7.66666651, 2.65028572,
                           2.98157120, 3.31285667, 3.64414287, 3.97542834, 4.30671406,
                           4.63799953, 4.96928549, 11.92628479, 12.42321396, 12.92014217,
                           13.41707039, 13.91399956, 14.41092777, 14.90785599, 15.40478516,
                           2.16437674, 2.43492365, 2.70547056, 2.97601795, 3.24656487,
                           3.51711202, 3.78765893, 4.05820608],
                          [1.58337951, 1.78130186, 1.97922409, 2.17714667, 2.37506914,
                           2.57299161, 2.77091384, 2.96883631, 1.89459133, 2.01300311,
                           2.13141513, 2.24982715, 2.36823893, 2.48665094, 2.60506320,
                           2.72347474, 1.89459133, 2.01300311, 2.13141513, 2.24982715,
                           2.36823893, 2.48665094, 2.60506320, 2.72347474, 3.43474555,
                           3.57786012, 3.72097445, 3.86408877, 4.00720310, 4.15031767,
                           4.29343224, 4.43654633]],
                tol=1e-4)
    return dict(forward=fwd, grad=grad)


def segment_formula():
    # core/kernels/segment_reduction_ali_ops_test.cc:75-240 (forward) and
    # :299-540 (grads).  input[i] = float(i/6) over 262144 x 6, indices = 2i,
    # segment_ids = i/2 for i < 131072.  ExpectTensorEqual (float: 4 ULP).
    rows, D, n = 262144, 6, 131072
    s = np.arange(65536, dtype=np.int64)
    base = (s * 4 + s * 4 + 2).astype(np.float32)
    r = np.arange(rows, dtype=np.int64)
    gmean = np.where(r % 2 == 0, (r // 4).astype(np.float32) / np.float32(2.0), 0.0).astype(np.float32)
    gsqrt = np.where(r % 2 == 0, (r // 4).astype(np.float32) / np.sqrt(np.float32(2.0)), 0.0).astype(np.float32)
    return dict(source="core/kernels/segment_reduction_ali_ops_test.cc:75-540",
                rows=rows, dim=D, n=n,
                note="expected values per output row (constant across the 6 columns)",
                forward_sum=base.tolist()[:64], forward_sum_formula="8*s+2",
                forward_mean_formula="(8*s+2)/2.0f", forward_sqrtn_formula="(8*s+2)/sqrtf(2.0f)",
                grad_mean_formula="even r: float(r/4)/2.0f else 0",
                grad_sqrtn_formula="even r: float(r/4)/sqrtf(2.0f) else 0",
                grad_mean_head=gmean.tolist()[:64], grad_sqrtn_head=gsqrt.tolist()[:64])


def ev_kats():
    # python/ops/embedding_variable_ops_test.py
    return dict(
        export=dict(source="python/ops/embedding_variable_ops_test.py:101-126",
                    dim=3, init=1.0, filter_freq=1, steps_to_live=10000,
                    lookup=[0, 1, 2, 5, 6, 7], runs=3,
                    keys=[0, 1, 2, 5, 6, 7], values=[[1.0] * 3] * 6,
                    versions=[0] * 6, freqs=[1] * 6),
        shape=dict(source="python/ops/embedding_variable_ops_test.py:128-141",
                   dim=3, lookup=[0, 1, 2, 5, 6, 7], expected=[6, 3]),
        counter_filter_gd=dict(source="python/ops/embedding_variable_ops_test.py:741-767",
                               dim=3, filter_freq=3, lr=0.1, key=1, loss_scale=2.0,
                               default_runs=3,
                               note="emb == 1.0 for the first 3 steps, != 1.0 at the 4th"),
        ev_equals_dense=dict(source="python/ops/embedding_variable_ops_test.py:825-997",
                             dim=3, init=1.0, ids=[0, 1, 2, 5, 6, 7], steps=5, lr=0.1,
                             loss_scale=2.0, optimizers=["sgd", "adagrad", "adam"],
                             adagrad_initial_accumulator=0.1,
                             adam=dict(beta1=0.9, beta2=0.999, epsilon=1e-8, delta=1e-5)),
    )


def fingerprint():
    """Fingerprint64 / StringToHashBucketFast KATs.  Byte strings are stored
    as generating rules (iota from a start byte, as the reference test builds
    them) or as literal ASCII."""
    return dict(
        # core/platform/fingerprint_test.cc:26-29
        fingerprint64=[dict(ascii="Hello", value=str(15404698994557526151)),
                       dict(ascii="World", value=str(18308117990299812472))],
        # python/kernel_tests/string_to_hash_bucket_op_test.py:40-50 (comments
        # give the raw fingerprints; num_buckets 10 -> [9, 2, 2, 5])
        fingerprint64_letters=[dict(ascii="a", value=str(12917804110809363939)),
                               dict(ascii="b", value=str(11795596070477164822)),
                               dict(ascii="c", value=str(11430444447143000872)),
                               dict(ascii="d", value=str(4470636696479570465))],
        hash_bucket_fast=dict(strings=["a", "b", "c", "d"], num_buckets=10,
                              expected=[9, 2, 2, 5]),
        # core/kernels/fingerprint_op_test.cc:64-74: uint8 [1, 3,4,5,6,7] iota
        # from 47 (wrapping), one row of 2520 bytes -> little-endian bytes
        op_bytes=dict(iota_start=47, length=2520, expected_le="2d90df0379363c43"),
        # :78-106: strings of 10, 7, 0, 19 bytes, iota from 0, 7, 71, 41; per
        # string fingerprints (shape {4}) and the fingerprint of their
        # concatenated little-endian bytes (shape {1, 2, 2})
        op_strings=dict(iota_starts=[0, 7, 71, 41], lengths=[10, 7, 0, 19],
                        expected_each_le=["eaffd6b2b24d709b", "6e9ded21c64a6152",
                                          "4f40902f3b6ae19a", "0d9b7f6323141cb8"],
                        expected_combined_le="92432852a37c4818"),
    )


def main():
    out = dict(fused_local=fused_local(), pre_lookup_partition=pre_lookup_partition(),
               post_lookup=post_lookup(),
               segment_formula=segment_formula(), ev=ev_kats(), fingerprint=fingerprint())
    for k, v in out.items():
        with open(os.path.join(HERE, k + ".json"), "w") as f:
            json.dump(v, f, indent=1)
    print("wrote", sorted(out))


if __name__ == "__main__":
    main()
