"""TP collective routing as pure functions: the RCCL
crossover that ``TPGroup.calibrate_collectives`` derives from its timing table, and the
per-message routing ``TPGroup._use_rccl`` applies — fed injected timing tables, so the
decisions the first 8-GPU run will take are pinned on the CPU. Also the env override and
the decode-size floor (decode messages never leave the in-house kernel)."""
import torch

from hipserve.parallel.comm import TPGroup, rccl_crossover, route_rccl

ROWS = [256, 512, 1024, 2048, 4096, 8192, 16384]


def table(car, rccl):
    return list(zip(ROWS, car, rccl))


def test_rccl_faster_everywhere():
    assert rccl_crossover(table([10] * 7, [5] * 7)) == 256


def test_rccl_never_faster():
    assert rccl_crossover(table([5] * 7, [10] * 7)) is None


def test_rccl_faster_from_a_size_on():
    car = [10, 20, 40, 80, 160, 320, 640]
    rccl = [30, 35, 45, 70, 120, 230, 450]
    assert rccl_crossover(table(car, rccl)) == 2048


def test_rccl_faster_only_at_some_sizes():
    # wins at 1024, loses at 2048, wins from 4096 on: one threshold, at 4096
    car = [10, 20, 40, 80, 160, 320, 640]
    rccl = [30, 35, 30, 90, 120, 230, 450]
    assert rccl_crossover(table(car, rccl)) == 4096
    # wins only in the middle: the largest size decides -> never
    rccl = [30, 15, 30, 60, 170, 330, 700]
    assert rccl_crossover(table(car, rccl)) is None


def test_ties_stay_in_house():
    assert rccl_crossover(table([10] * 7, [10] * 7)) is None


def test_unsorted_results():
    res = list(reversed(table([10, 20, 40, 80, 160, 320, 640], [30, 35, 45, 70, 120, 230, 450])))
    assert rccl_crossover(res) == 2048


def test_route_rccl():
    assert route_rccl(8192, 2048, 512, "nccl", False)
    assert route_rccl(2048, 2048, 512, "nccl", False)
    assert not route_rccl(1024, 2048, 512, "nccl", False)       # below the crossover
    assert not route_rccl(8192, None, 512, "nccl", False)       # not calibrated / never faster
    assert not route_rccl(8192, 2048, 512, "gloo", False)       # gloo group (shared-GPU tests)
    assert not route_rccl(8192, 2048, 512, "nccl", True)        # inside a hipGraph capture
    # crossover below the decode floor: decode-sized messages stay in-house
    assert not route_rccl(256, 128, 512, "nccl", False)
    assert not route_rccl(512, 128, 512, "nccl", False)
    assert route_rccl(513, 128, 512, "nccl", False)


def test_group_routing_and_env_override(monkeypatch):
    g = TPGroup(0, 2, None, torch.device("cpu"))
    g.backend = "nccl"
    g.rccl_min_rows = 1024
    g.rccl_floor_rows = 256
    assert g._use_rccl(4096) and not g._use_rccl(512)
    # the env override short-circuits calibration, -1 = never
    g.custom_ar = object()
    monkeypatch.setenv("HIPSERVE_CAR_RCCL_MIN_ROWS", "-1")
    assert g.calibrate_collectives(4096, 8192) == [] and g.rccl_min_rows is None
    monkeypatch.setenv("HIPSERVE_CAR_RCCL_MIN_ROWS", "3000")
    g.calibrate_collectives(4096, 8192)
    assert g.rccl_min_rows == 3000 and g._use_rccl(3000) and not g._use_rccl(2999)
