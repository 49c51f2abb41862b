"""Host check of the wave edge kernel's slot-range split (csrc/edge_wave.hip,
csrc/layer.hip prep): wave w walks slots [w S / G, (w + 1) S / G); the unit a
wave starts inside a tile goes to side[w]; the node stage adds, for tile t, the
side blocks of the ranks lo..hi given in closed form.  Brute force over many
(ntiles, k, G): every slot of every tile is summed exactly once, in slot order."""
import pytest


def closed_form(t, k, G, S):
    lo = max(((t * k + 1) * G + S - 1) // S, 1)
    hi = min(((t + 1) * k * G + S - 1) // S - 1, G - 1)
    return lo, hi


def units(ntiles, k, G):
    """(tile, first slot, last slot + 1, destination) of every unit, wave by wave."""
    S = ntiles * k
    out = []
    for w in range(G):
        s0, s1 = w * S // G, (w + 1) * S // G
        s = s0
        while s < s1:
            t = s // k
            e = min(s1, (t + 1) * k)
            dest = ("side", w) if (s == s0 and s0 % k) else ("out", t)
            out.append((t, s, e, dest))
            s = e
    return out


@pytest.mark.parametrize("ntiles,k,G", [(2521, 35, 1024), (7, 35, 20), (7, 1, 7), (7, 3, 20),
                                        (316, 35, 945), (1, 35, 35), (3, 35, 6), (576, 35, 1024),
                                        (100, 8, 1024), (5, 4, 19)])
def test_slot_split_covers_every_slot_once(ntiles, k, G):
    S = ntiles * k
    G = min(G, S)
    us = units(ntiles, k, G)
    per_tile = {}
    for t, s, e, dest in us:
        per_tile.setdefault(t, []).append((s, e, dest))
    for t in range(ntiles):
        parts = sorted(per_tile[t])
        # contiguous cover of [t k, (t + 1) k), in slot order
        assert parts[0][0] == t * k and parts[-1][1] == (t + 1) * k
        assert all(a[1] == b[0] for a, b in zip(parts, parts[1:]))
        # exactly one part stored to the tile's own rows: the one starting at its first slot
        assert parts[0][2] == ("out", t)
        assert all(p[2][0] == "side" for p in parts[1:])
        # the node stage's closed-form rank range names exactly those side blocks, in order
        lo, hi = closed_form(t, k, G, S)
        assert [p[2][1] for p in parts[1:]] == list(range(lo, hi + 1))
