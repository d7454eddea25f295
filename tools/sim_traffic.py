#!/usr/bin/env python3
"""Memory-traffic model of the round split kernel for alternative row layouts.

Trains the headline configuration on the CPU learner (rows scaled down; densities, not row
counts, decide the line waste), walks every accepted split of a few trees and counts, per
expanded node, the distinct L2 lines a design touches:

  index   : the current design -- row indices in leaf order (ascending runs), row-major bins and
            (g, h) in original row order: index read/write streams, split-column byte, and the
            smaller child's 28-B row + 8-B (g, h) gathered by index
  ordered : every node's rows materialised in leaf order (bins + (g, h) + index): the parent is
            read and both children written as streams, the histogram reads nothing extra
  gh      : leaf-ordered (g, h) copy beside the index, bins gathered by index

  python tools/sim_traffic.py --rows 2000000 --iters 30 --line 128
"""
import argparse
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def lines(addr_lo, nbytes, line):
    """distinct lines touched by [addr_lo, addr_lo + nbytes) for every element (sorted unique)"""
    a = addr_lo // line
    b = (addr_lo + nbytes - 1) // line
    if np.array_equal(a, b):
        return np.unique(a).size
    return np.unique(np.concatenate([a, b])).size


def node_rows(tree, leaf_of_row):
    """{internal node index: ascending row array} from a dumped tree and per-row leaf ids"""
    order = np.argsort(leaf_of_row, kind="stable")
    bounds = np.searchsorted(leaf_of_row[order], np.arange(leaf_of_row.max() + 2))
    out = []

    def walk(n, depth):
        if "leaf_index" in n:
            li = n["leaf_index"]
            return order[bounds[li]:bounds[li + 1]]
        left = walk(n["left_child"], depth + 1)
        right = walk(n["right_child"], depth + 1)
        rows = np.sort(np.concatenate([left, right]))
        out.append((depth, rows, left if left.size <= right.size else right))
        return rows

    walk(tree["tree_structure"], 0)
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, default=2_000_000)
    ap.add_argument("--iters", type=int, default=30)
    ap.add_argument("--line", type=int, default=128)
    ap.add_argument("--trees", default="0,10,-1")
    ap.add_argument("--row-bytes", type=int, default=28)
    args = ap.parse_args()
    import lightgbmv1_amd as lgb
    from bench import make_rows
    X, y = make_rows(0, args.rows, 28)
    params = {"objective": "binary", "max_bin": 255, "num_leaves": 63, "learning_rate": 0.1, "min_data_in_leaf": 1,
              "min_sum_hessian_in_leaf": 100, "verbose": -1, "device_type": "cpu"}
    bst = lgb.train(params, lgb.Dataset(X, y, params=params), args.iters)
    dump = bst.dump_model()
    leaves = bst.predict(X, pred_leaf=True)
    L, RB = args.line, args.row_bytes
    for t in [int(s) for s in args.trees.split(",")]:
        ti = t % bst.num_trees()
        tree = dump["tree_info"][ti]
        nodes = node_rows(tree, np.asarray(leaves[:, ti], dtype=np.int64))
        tot = {"index": 0, "ordered": 0, "gh": 0}
        parts = {"idx": 0, "col": 0, "rowg": 0, "ghg": 0}
        visits = hist = 0
        by_depth = {}
        for depth, rows, h in nodes:
            n = rows.size
            visits += n
            hist += h.size
            idx = 8 * n
            col = lines(rows, 1, L) * L
            rowg = lines(h * RB, RB, L) * L
            ghg = lines(h * 8, 8, L) * L
            parts["idx"] += idx
            parts["col"] += col
            parts["rowg"] += rowg
            parts["ghg"] += ghg
            cur = idx + col + rowg + ghg
            tot["index"] += cur
            tot["ordered"] += 2 * (RB + 8 + 4) * n
            tot["gh"] += idx + 16 * n + col + rowg
            d = by_depth.setdefault(depth, [0, 0, 0])
            d[0] += n
            d[1] += cur
            d[2] += 2 * (RB + 8 + 4) * n
        scale = 10_000_000 / args.rows
        print("tree %d: %d splits, parent-row visits %.2f x N, hist rows %.2f x N" % (ti, len(nodes), visits / args.rows, hist / args.rows))
        for k, v in tot.items():
            print("  %-8s %.2f GB/tree at 10M rows (%.1f B per visit)" % (k, v * scale / 1e9, v / visits))
        print("  index parts (B/visit): " + ", ".join("%s %.1f" % (k, v / visits) for k, v in parts.items()))
        for depth in sorted(by_depth):
            n, c, o = by_depth[depth]
            print("    depth %2d: visits %.2f x N, index %.1f B/visit, ordered %.1f" % (depth, n / args.rows, c / n, o / n))


if __name__ == "__main__":
    main()
