"""Known-answer tests restated from the reference's own suites, run through
the product on the CPU (host C++ of libradler_amd via the `radler` module):

* cpp/math/test/test_dijkstra_splitter.cc:92-538 — DivideVertically /
  DivideHorizontally (free and constrained), AddVertical/HorizontalDivider +
  FloodVertical/HorizontalArea, GetBoundingMask (incl. the even-size
  extension), and the noise partition property.
* cpp/test/test_component_list.cc:11-105 — Add / MergeDuplicates /
  GetComponent / GetPositions / MultiplyScaleComponent, plus the merge rules
  of component_list.h:222-263 (zero sums vanish, per-frequency emission order).

The splitter's oracle restatement (oracle/tiling.cc) matches the product on
random images (tests/test_tiling.py), so these vectors pin both.
"""
import numpy as np
import pytest

from radler_import import radler as rd

T = rd.tiling


def make_image(width, rows):
    s = "".join(rows)
    h = len(s) // width
    assert width * h == len(s)
    return np.array([[0.1 if s[x + y * width] == "X" else 10.0 for x in range(width)]
                     for y in range(h)], np.float32)


def path_str(img):
    return ["".join(" " if v == 0.0 else "X" for v in row) for row in img]


def mask_str(mask, width):
    m = np.asarray(mask).reshape(-1, width)
    return ["".join("X" if v else " " for v in row) for row in m]


def column_str(img, x):
    return "".join(" " if v == 10.0 else "X" for v in img[:, x])


def row_str(img, y):
    return "".join(" " if v == 10.0 else "X" for v in img[y])


def test_vertical():  # :92-119
    image = make_image(10, ["X         ", " X        ", "  X       ", "   XXX    ",
                            "     X    ", "         X", "   X      ", "    XXXX  ",
                            "        X ", "      XX  "])
    out = np.zeros_like(image)
    T.divide_vertically(image, out, 0, 10)
    assert path_str(out) == ["X         ", " X        ", "  X       ", "   XX     ",
                             "     X    ", "    X     ", "   X      ", "    XXXX  ",
                             "        X ", "       X  "]


def test_vertical_constrained():  # :121-153
    image = make_image(10, [" X  X     ", " X        ", "  X       ", "   XXX    ",
                            "     X    ", "XX       X", "  XX      ", "    XXXX  ",
                            "        X ", "      XX  "])
    out = image.copy()
    T.divide_vertically(image, out, 2, 8)
    assert path_str(out) == ["XX  X   XX", "XX X    XX", "XXX     XX", "XX XX   XX",
                             "XX   X  XX", "XX  X   XX", "XX X    XX", "XX  X   XX",
                             "XX   X  XX", "XX    X XX"]
    assert column_str(out, 0) == "     X    "
    assert column_str(out, 1) == "XX   X    "
    assert column_str(out, 8) == "        X "
    assert column_str(out, 9) == "     X    "


def test_horizontal():  # :155-182
    image = make_image(10, ["    X     ", "          ", "  X       ", "   XXXXXX ",
                            "     X    ", " X   X   X", " X    X   ", " X     X  ",
                            " X      X ", "X     XX X"])
    out = np.zeros_like(image)
    T.divide_horizontally(image, out, 0, 10)
    assert path_str(out) == ["          ", "          ", "          ", "   XX     ",
                             "  X  X    ", " X   X    ", " X    X   ", " X     X  ",
                             " X      X ", "X        X"]


def test_horizontal_constrained():  # :184-216
    image = make_image(10, ["  XXX     ", " XXXXXX   ", " X     XXX", "X   XXX   ",
                            "   XX     ", "X        X", "XX        ", "  X      X",
                            "   XXXXXX ", "    XXXX  "])
    out = image.copy()
    T.divide_horizontally(image, out, 2, 8)
    assert path_str(out) == ["XXXXXXXXXX", "XXXXXXXXXX", " X     XXX", "X X XXX   ",
                             "   X      ", "          ", "          ", "          ",
                             "XXXXXXXXXX", "XXXXXXXXXX"]
    assert row_str(out, 0) == "  XXX     "
    assert row_str(out, 1) == " XXXXXX   "
    assert row_str(out, 8) == "   XXXXXX "
    assert row_str(out, 9) == "    XXXX  "


def test_flood_vertical_area():  # :218-277
    w = h = 9
    image = make_image(w, ["   X     ", "    X    ", "    X    ", "   X     ", "  X      ",
                           "   XXX   ", "      X  ", "      X  ", "      X  "])
    scratch, lines = image.copy(), np.zeros_like(image)
    T.add_vertical_divider(image, scratch, lines, 2, 7)
    assert path_str(lines) == ["   X     ", "    X    ", "    X    ", "   X     ",
                               "  X      ", "   XXX   ", "      X  ", "      X  ",
                               "      X  "]
    mask = np.zeros((h, w), bool)
    assert T.flood_vertical_area(lines, 1, mask) == (0, 6)
    assert mask_str(mask, w) == ["XXX      ", "XXXX     ", "XXXX     ", "XXX      ",
                                 "XX       ", "XXX      ", "XXXXXX   ", "XXXXXX   ",
                                 "XXXXXX   "]
    assert T.flood_vertical_area(lines, 7, mask) == (2, 7)
    assert mask_str(mask, w) == ["   XXXXXX", "    XXXXX", "    XXXXX", "   XXXXXX",
                                 "  XXXXXXX", "   XXXXXX", "      XXX", "      XXX",
                                 "      XXX"]


def test_flood_horizontal_area():  # :279-335
    w, h = 10, 8
    image = make_image(w, ["          ", "          ", "  XX    XX", " X  X  X  ",
                           " X   X X  ", " X   X X  ", "X     X   ", "          "])
    scratch, lines = image.copy(), np.zeros_like(image)
    T.add_horizontal_divider(image, scratch, lines, 2, 7)
    assert path_str(lines) == ["          ", "          ", "  XX    XX", " X  X  X  ",
                               " X   X X  ", " X   X X  ", "X     X   ", "          "]
    mask = np.zeros((h, w), bool)
    assert T.flood_horizontal_area(lines, 1, mask) == (0, 6)
    assert mask_str(mask, w) == ["XXXXXXXXXX", "XXXXXXXXXX", "XX  XXXX  ", "X    XX   ",
                                 "X     X   ", "X     X   ", "          ", "          "]
    assert T.flood_horizontal_area(lines, 7, mask) == (2, 6)
    assert mask_str(mask, w) == ["          ", "          ", "  XX    XX", " XXXX  XXX",
                                 " XXXXX XXX", " XXXXX XXX", "XXXXXXXXXX", "XXXXXXXXXX"]


def test_get_bounding_mask():  # :337-489
    w, h = 10, 8
    image = make_image(w, ["    X     "] * 4 + ["XXXXXXXXXX"] + ["    X     "] * 3)
    lines = np.zeros_like(image)
    T.divide_vertically(image, lines, 3, 6)
    mask = np.zeros((h, w), bool)
    xl, wl = T.flood_vertical_area(lines, 1, mask)
    assert (xl, wl) == (0, 4)
    mask_l = np.ascontiguousarray(mask[:, xl:xl + wl])
    assert mask_str(mask_l, wl) == ["XXXX", "XXXX", "XXXX", "XXXX", "XXX ", "XXXX",
                                    "XXXX", "XXXX"]
    xr, wr = T.flood_vertical_area(lines, 7, mask)
    assert (xr, wr) == (3, 7)
    mask_r = np.ascontiguousarray(mask[:, xr:xr + wr])
    assert mask_str(mask_r, wr) == [" XXXXXX"] * 4 + ["XXXXXXX"] + [" XXXXXX"] * 3

    lines[:] = 0.0
    T.divide_horizontally(image, lines, 3, 6)
    assert T.flood_horizontal_area(lines, 1, mask) == (0, 4)
    assert mask_str(mask, w) == ["XXXXXXXXXX"] * 3 + ["XXXX XXXXX"] + [" " * 10] * 4

    out = np.zeros((h, w), bool)
    assert T.get_bounding_mask(w, h, mask_l, xl, wl, mask, out) == (0, 0, 4, 4)
    assert mask_str(out, w) == ["XXXX      "] * 4 + [" " * 10] * 4
    out[:] = False
    assert T.get_bounding_mask(w, h, mask_r, xr, wr, mask, out) == (4, 0, 6, 4)
    assert mask_str(out, w) == ["    XXXXXX"] * 3 + ["     XXXXX"] + [" " * 10] * 4

    assert T.flood_horizontal_area(lines, 7, mask) == (3, 5)
    out[:] = False
    assert T.get_bounding_mask(w, h, mask_l, xl, wl, mask, out) == (0, 4, 4, 4)
    assert mask_str(out, w) == [" " * 10] * 4 + ["XXX       "] + ["XXXX      "] * 3
    out[:] = True
    # odd width and height grow by one; at the far right/bottom the box moves
    # left/up instead (:467-470)
    assert T.get_bounding_mask(w, h, mask_r, xr, wr, mask, out) == (2, 2, 8, 6)
    assert mask_str(out, w) == ["XXX       ", "XXX       ", "XX        ", "XX  X     ",
                                "XX XXXXXXX", "XX  XXXXXX", "XX  XXXXXX", "XX  XXXXXX"]


def test_get_bounding_mask_on_noise():  # :491-538 (100 of its 1000 repeats)
    """The four quadrant masks partition the image."""
    w = h = 80
    rng = np.random.default_rng(0)
    for _ in range(100):
        image = rng.standard_normal((h, w)).astype(np.float32)
        lv, lh = np.zeros_like(image), np.zeros_like(image)
        T.divide_vertically(image, lv, w // 4, w * 3 // 4)
        T.divide_horizontally(image, lh, h // 4, h * 3 // 4)
        ml, mr, mt, mb = (np.zeros((h, w), bool) for _ in range(4))
        T.flood_vertical_area(lv, w // 8, ml)
        T.flood_vertical_area(lv, w * 7 // 8, mr)
        T.flood_horizontal_area(lh, w // 8, mt)
        T.flood_horizontal_area(lh, w * 7 // 8, mb)
        count = np.zeros((h, w), int)
        for vm, hm in ((ml, mt), (mr, mt), (ml, mb), (mr, mb)):
            out = np.zeros((h, w), bool)
            T.get_bounding_mask(w, h, vm, 0, w, hm, out)
            count += out
        assert (count == 1).all()


@pytest.fixture
def component_list():  # test_component_list.cc:11-27
    cl = rd.ComponentList(512, 512, 4, 3)
    cl.add(256, 256, 1, [1.0, 2.0, 3.0])
    cl.add(256, 256, 1, [5.0, 6.0, 7.0])
    cl.add(511, 511, 0, [8.0, 9.0, 10.0])
    cl.add(13, 42, 3, [11.0, 12.0, 13.0])
    cl.merge_duplicates()
    return cl


def test_component_list_adding_values(component_list):  # :29-59
    cl = component_list
    assert [cl.component_count(s) for s in range(4)] == [1, 1, 0, 1]
    assert cl.get_component(0, 0) == (511, 511, [8.0, 9.0, 10.0])
    assert cl.get_component(1, 0) == (256, 256, [6.0, 8.0, 10.0])
    assert cl.get_component(3, 0) == (13, 42, [11.0, 12.0, 13.0])


def test_component_list_get_position(component_list):  # :61-75
    cl = component_list
    assert [len(cl.get_positions(s)) for s in range(4)] == [1, 1, 0, 1]
    assert cl.get_positions(0)[0] == (511, 511)
    assert cl.get_positions(1)[0] == (256, 256)
    assert cl.get_positions(3)[0] == (13, 42)


def test_component_list_multiply_scale_component(component_list):  # :77-105
    cl = component_list
    for s in (0, 1, 3):
        for f in range(cl.n_frequencies):
            cl.multiply_scale_component(s, 0, f, float(f + 1))
    assert cl.get_component(0, 0)[2] == [8.0, 18.0, 30.0]
    assert cl.get_component(1, 0)[2] == [6.0, 16.0, 30.0]
    assert cl.get_component(3, 0)[2] == [11.0, 24.0, 39.0]


def test_component_list_merge_rules():
    """component_list.h:222-263: summed values of a position that cancel in
    every frequency drop the position; the output lists, frequency by
    frequency, the raster positions whose value is non-zero there."""
    cl = rd.ComponentList(8, 8, 1, 2)
    cl.add(5, 1, 0, [1.0, 2.0])
    cl.add(5, 1, 0, [-1.0, -2.0])   # cancels: vanishes
    cl.add(3, 6, 0, [0.0, 4.0])     # zero in frequency 0: emitted second
    cl.add(7, 2, 0, [3.0, 0.0])
    cl.add(2, 0, 0, [0.5, 0.5])
    cl.add(7, 2, 0, [1.0, 1.0])
    cl.merge_duplicates()
    got = [cl.get_component(0, i) for i in range(cl.component_count(0))]
    assert got == [(2, 0, [0.5, 0.5]), (7, 2, [4.0, 1.0]), (3, 6, [0.0, 4.0])]
