"""ResNet-18 (group size g, average terms alpha) grid -- the reference's
evaluate_group_size.py (evaluate_group_size.py:1-91), same CLI and result JSON.

    python evaluate_group_size.py <val_dir> -a resnet18
    torchrun --nproc-per-node 8 evaluate_group_size.py --synthetic -a resnet18
    torchrun --nproc-per-node 2 evaluate_group_size.py --synthetic -a resnet18 --gpu -1  # CPU

Each of the 25 settings is evaluated batch-sharded over all ranks; the
results JSON does not depend on the world size.
"""
import evaluate_cnn
from evaluate_cnn import build_parser, eval_model, save, setup

AVG_TERM_SETTINGS = [1.0, 1.25, 1.5, 2.0, 3.0]
GROUP_SIZES = [1, 2, 8, 16, 32]


def main(argv=None):
    args = build_parser().parse_args(argv)
    model = setup(args)

    results = {}

    # Term Revealing Settings (evaluate_group_size.py:71-88)
    weight_bits = 9
    group_size = 8
    data_bits = 9
    data_terms = 3
    for group_size in GROUP_SIZES:
        key = str(group_size)
        results[key] = {'avg_terms': [], 'accs': [], 'tmacs': []}
        for avg_term in AVG_TERM_SETTINGS:
            weight_terms = round(avg_term * group_size)
            res = eval_model(args, model, weight_bits, group_size,
                             weight_terms, data_bits, data_terms)
            acc, tmacs, avg_term, params = res
            print(data_terms, weight_terms, tmacs, acc)
            results[key]['accs'].append(acc)
            results[key]['tmacs'].append(tmacs)
            results[key]['avg_terms'].append(avg_term)

    save(args, results, '{}-group-size-results.json'.format(args.arch))
    evaluate_cnn.finish()
    return results


if __name__ == '__main__':
    main()
