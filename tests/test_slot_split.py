"""Host check of the wave edge kernel's work split (csrc/edge_wave.hip,
csrc/layer.hip prep, layer.hpp EdgeSplit / edge_wave_plan), restated in Python:
a segment's S = ntiles * k neighbour slots are cut into U summation units
(unit u = slots [u S / U, (u + 1) S / U)); wave j walks units [j m, (j + 1) m);
a run (the part of a unit inside one tile) closes at its tile's end, at a unit
boundary and at the wave's end; a run that starts a tile goes to out, a run
that starts at a unit boundary inside a tile to side[u]; the node stage adds,
for tile t, the side blocks of the units lo..hi given in closed form.  Brute
force over many (ntiles, k, U, m): every slot of every tile is summed exactly
once, in slot order, and the runs -- hence the summation order -- depend on
(S, U) only, not on how many units a wave takes."""
import pytest


def closed_form(t, k, U, S):
    lo = max(((t * k + 1) * U + S - 1) // S, 1)
    hi = min(((t + 1) * k * U + S - 1) // S - 1, U - 1)
    return lo, hi


def plan(nseg, S_seg, cus=256, side_cap=1 << 40):
    """edge_wave_plan (edge_wave.hip): (U, m, waves)."""
    u0 = 1
    while u0 * 2 * 44 <= S_seg:
        u0 *= 2
    u1 = max(4 * cus // nseg, 1)
    m = -(-u0 // u1)
    U = u1 * m
    cap = min(S_seg, side_cap // nseg)
    if U > cap:
        U, m = max(cap, 1), 1
    return U, m, nseg * (U // m)


def runs(ntiles, k, U, m):
    """(tile, first slot, last slot + 1, destination) of every run, as the
    kernel's slot stream produces them, wave by wave."""
    S = ntiles * k
    out = []
    for j in range(-(-U // m)):
        u_end = min((j + 1) * m, U)
        s0, s1 = j * m * S // U, u_end * S // U
        u_next = j * m + 1
        ub = u_next * S // U if u_next < u_end else s1
        run_side = j * m if s0 % k else -1
        s, start = s0, s0
        while s < s1:
            new_unit = s + 1 == ub
            close = (s % k) + 1 == k or s + 1 == s1 or new_unit
            if close:
                dest = ("out", s // k) if run_side < 0 else ("side", run_side)
                out.append((s // k, start, s + 1, dest))
                start = s + 1
                run_side = u_next if new_unit and (s + 1) % k else -1
                if new_unit:
                    u_next += 1
                    ub = u_next * S // U if u_next < u_end else s1
            s += 1
    return out


@pytest.mark.parametrize("ntiles,k,U,m", [(158, 35, 64, 1), (158, 35, 64, 2), (158, 35, 128, 4),
                                          (7, 35, 20, 1), (7, 1, 7, 1), (7, 3, 20, 3),
                                          (316, 35, 945, 1), (1, 35, 35, 5), (3, 35, 6, 2),
                                          (576, 35, 1024, 1), (100, 8, 512, 8), (5, 4, 19, 1)])
def test_runs_cover_every_slot_once(ntiles, k, U, m):
    S = ntiles * k
    U = min(U, S)
    if U % m:
        pytest.skip("U must be a multiple of m")
    rs = runs(ntiles, k, U, m)
    per_tile = {}
    for t, s, e, dest in rs:
        per_tile.setdefault(t, []).append((s, e, dest))
    for t in range(ntiles):
        parts = sorted(per_tile[t])
        # contiguous cover of [t k, (t + 1) k), in slot order
        assert parts[0][0] == t * k and parts[-1][1] == (t + 1) * k
        assert all(a[1] == b[0] for a, b in zip(parts, parts[1:]))
        # exactly one part stored to the tile's own rows: the one starting at its first slot
        assert parts[0][2] == ("out", t)
        assert all(p[2][0] == "side" for p in parts[1:])
        # the node stage's closed-form unit range names exactly those side blocks, in order
        lo, hi = closed_form(t, k, U, S)
        assert [p[2][1] for p in parts[1:]] == list(range(lo, hi + 1))


@pytest.mark.parametrize("ntiles,k,U", [(158, 35, 64), (144, 35, 64), (100, 8, 256)])
def test_runs_do_not_depend_on_units_per_wave(ntiles, k, U):
    base = sorted(runs(ntiles, k, U, 1))
    for m in (2, 4, 8):
        if U % m == 0:
            assert sorted(runs(ntiles, k, U, m)) == base


def test_plan_fills_the_chip_and_is_shared_by_power_of_two_batches():
    S_cy = 158 * 35                       # cylinder: 2521 nodes, k = 35
    for nseg in (1, 2, 4, 8, 16, 32, 64, 128):
        U, m, waves = plan(nseg, S_cy)
        assert U % m == 0 and waves == nseg * U // m
        assert waves == 1024                # one wave per SIMD on 256 CUs
    # 16 and more trajectories share U (the same summation order for every row)
    assert len({plan(nseg, S_cy)[0] for nseg in (16, 32, 64, 128)}) == 1
    # other counts still fill the chip to within one unit
    for nseg in (3, 5, 12, 24):
        U, m, waves = plan(nseg, S_cy)
        assert waves <= 1024 and U % m == 0
