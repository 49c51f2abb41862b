"""Host check of the wave edge kernel's work split (csrc/edge_wave.hip,
csrc/layer.hip prep, layer.hpp EdgeSplit / edge_wave_plan), restated in Python:
a segment's S = ntiles * k neighbour slots are cut into U summation units
(unit u = slots [u S / U, (u + 1) S / U)); wave j of the w waves of a segment
walks units [j U / w, (j + 1) U / w);
a run (the part of a unit inside one tile) closes at its tile's end, at a unit
boundary and at the wave's end; a run that starts a tile goes to out, a run
that starts at a unit boundary inside a tile to side[u]; the node stage adds,
for tile t, the side blocks of the units lo..hi given in closed form.  Brute
force over many (ntiles, k, U, w): every slot of every tile is summed exactly
once, in slot order, and the runs -- hence the summation order -- depend on
(S, U) only, not on how many units a wave takes; U depends on the segment
alone, so any shard of a batch sums every row in the same order."""
import pytest


def closed_form(t, k, U, S):
    lo = max(((t * k + 1) * U + S - 1) // S, 1)
    hi = min(((t + 1) * k * U + S - 1) // S - 1, U - 1)
    return lo, hi


K_WAVE_TILES = 64   # layer.hpp kWaveTiles: a wave's row split scales live in LDS


def plan(nseg, S_seg, cus=256, side_cap=1 << 40, k=35):
    """edge_wave_plan (edge_wave.hip): (U, waves per segment, waves)."""
    U = 1
    while U * 2 * 22 <= S_seg:
        U *= 2
    if S_seg >= 16384:                    # one segment fills the chip alone
        while U < 1024 and U * 2 * 11 <= S_seg:
            U *= 2
    cap = min(S_seg, side_cap // nseg)
    if U > cap:
        U = max(cap, 1)
    w = min(max(4 * cus // nseg, 1), U)
    spu = -(-S_seg // U)

    def tiles_of(ww):
        return (-(-U // ww) * spu + k - 1) // k + 1

    while w < U and tiles_of(w) > K_WAVE_TILES:
        w = min(2 * w, U)
    assert tiles_of(w) <= K_WAVE_TILES
    return U, w, nseg * w


def tiles_spanned(ntiles, k, U, w):
    """Largest number of tiles one wave's slot range touches."""
    S = ntiles * k
    most = 0
    for j in range(w):
        s0, s1 = (j * U // w) * S // U, ((j + 1) * U // w) * S // U
        if s0 < s1:
            most = max(most, (s1 - 1) // k - s0 // k + 1)
    return most


def runs(ntiles, k, U, w):
    """(tile, first slot, last slot + 1, destination) of every run, as the
    kernel's slot stream produces them, wave by wave (w waves)."""
    S = ntiles * k
    out = []
    for j in range(w):
        u_begin, u_end = j * U // w, (j + 1) * U // w
        s0, s1 = u_begin * S // U, u_end * S // U
        if s0 >= s1:
            continue
        u_next = u_begin + 1
        ub = u_next * S // U if u_next < u_end else s1
        run_side = u_begin if s0 % k else -1
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


@pytest.mark.parametrize("ntiles,k,U,w", [(158, 35, 64, 64), (158, 35, 128, 64), (158, 35, 128, 85),
                                          (158, 35, 128, 42), (7, 35, 20, 20), (7, 1, 7, 7), (7, 3, 20, 7),
                                          (316, 35, 945, 945), (1, 35, 35, 7), (3, 35, 6, 3),
                                          (576, 35, 1024, 1024), (100, 8, 512, 64), (5, 4, 19, 19),
                                          (144, 35, 128, 32), (158, 35, 128, 1)])
def test_runs_cover_every_slot_once(ntiles, k, U, w):
    S = ntiles * k
    U = min(U, S)
    w = min(w, U)
    rs = runs(ntiles, k, U, w)
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


@pytest.mark.parametrize("ntiles,k,U", [(158, 35, 128), (144, 35, 128), (100, 8, 256)])
def test_runs_do_not_depend_on_waves_per_segment(ntiles, k, U):
    base = sorted(runs(ntiles, k, U, U))
    for w in (1, 3, 16, 42, 64, 85, U // 2):
        assert sorted(runs(ntiles, k, U, w)) == base


def test_plan_is_segment_only_and_fills_the_chip():
    S_cy = 158 * 35                       # cylinder: 2521 nodes, k = 35
    S_bu = 144 * 35                       # Burgers 48 x 48: 2304 nodes
    for S in (S_cy, S_bu):
        # every segment count sums a row in the same order (U from the segment alone)
        assert len({plan(nseg, S)[0] for nseg in range(1, 129)}) == 1
    assert plan(16, S_cy)[0] == 128 and plan(32, S_bu)[0] == 128
    for nseg in (8, 16, 32, 64, 128):      # power-of-two shards: one wave per SIMD
        assert plan(nseg, S_cy)[2] == 1024
    for nseg in (3, 5, 12, 24):            # others: never more waves than SIMDs
        U, w, waves = plan(nseg, S_cy)
        assert waves <= 1024 and w <= U
    # the side-block cap (3 seg_n / 16 blocks per segment) is a function of the segment
    assert plan(16, 5530, side_cap=16 * (3 * 2521 // 16))[0] == 128
    # a 96 x 96 Burgers trajectory (576 tiles x 35 slots) alone: 1024 units of
    # 19-20 slots, one wave per SIMD (512 units with the 22-44 rule alone)
    S_96 = 576 * 35
    assert plan(1, S_96, side_cap=3 * 9216 // 16) == (1024, 1024, 1024)
    assert len({plan(nseg, S_96)[0] for nseg in range(1, 9)}) == 1


@pytest.mark.parametrize("nseg,ntiles,k", [(16, 158, 35), (2048, 158, 35), (4096, 144, 35), (1, 65536, 35),
                                           (3000, 300, 8), (1, 1 << 20, 35)])
def test_plan_keeps_a_wave_within_its_lds_tiles(nseg, ntiles, k):
    """Many segments (one wave per segment by the SIMD count) or one huge
    segment: the plan adds waves until none spans more than kWaveTiles tiles
    (its row split scales are computed once into LDS); U, hence every sum,
    is unchanged."""
    S = ntiles * k
    U, w, waves = plan(nseg, S, side_cap=nseg * 3 * ntiles, k=k)
    U0 = plan(1, S, side_cap=3 * ntiles, k=k)[0]
    assert U == U0
    assert tiles_spanned(ntiles, k, U, w) <= K_WAVE_TILES
