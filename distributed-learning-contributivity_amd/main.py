"""Command-line entry point - drop-in for the reference's main.py (same flags, same results.csv).

    python main.py -f config.yml [-v]

Reads the experiment YAML (mplc/utils.py schema), validates every scenario (instantiate + split, no
training), then for each repeat and scenario runs the multi-partner learning and the contributivity
methods on the MI355X engine and appends the scenario's to_dataframe() rows (plus random_state and
scenario_id) to <experiment_path>/results.csv, header only once (main.py:44-107 of the reference).
Under torch.distributed (one process per GPU) coalition trainings are sharded over the ranks and only
rank 0 writes results.csv.
"""
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
if HERE not in sys.path:
    sys.path.insert(0, HERE)

from mplc import scenario, utils  # noqa: E402

DEFAULT_CONFIG_FILE = "./config.yml"


def validate_scenario_list(scenario_params_list, experiment_path):
    """Instantiate every scenario and split its data without training (main.py:110-130)."""
    for scenario_params in scenario_params_list:
        sc = scenario.Scenario(**scenario_params, experiment_path=experiment_path, is_dry_run=True)
        sc.instantiate_scenario_partners()
        if sc.samples_split_type == "basic":
            sc.split_data(is_logging_enabled=False)
        else:
            raise NotImplementedError("the advanced split is outside the engine's scope (DESIGN.md)")


def _rank():
    try:
        import torch.distributed as dist
        if dist.is_available() and dist.is_initialized():
            return dist.get_rank()
    except Exception:  # noqa: BLE001
        pass
    return 0


def main(argv=None):
    args = utils.parse_command_line_arguments(argv)
    utils.init_logger(args.verbose)
    config_file = args.file or DEFAULT_CONFIG_FILE
    utils.logger.info(f"Using config file: {config_file}")
    config = utils.get_config_from_file(config_file)
    scenario_params_list = utils.get_scenario_params_list(config["scenario_params_list"])
    experiment_path = config["experiment_path"]
    n_repeats = config["n_repeats"]
    validate_scenario_list(scenario_params_list, experiment_path)
    utils.set_log_file(experiment_path)
    utils.init_gpu_config()
    for i in range(n_repeats):
        utils.logger.info(f"Repeat {i + 1}/{n_repeats}")
        for scenario_id, scenario_params in enumerate(scenario_params_list):
            utils.logger.info(f"Scenario {scenario_id + 1}/{len(scenario_params_list)}: {scenario_params}")
            current = scenario.Scenario(**scenario_params, experiment_path=experiment_path,
                                        scenario_id=scenario_id + 1, repeats_count=i + 1)
            current.run()
            df = current.to_dataframe()
            df["random_state"] = i
            df["scenario_id"] = scenario_id
            if _rank() == 0:
                with open(experiment_path / "results.csv", "a") as f:
                    df.to_csv(f, header=f.tell() == 0, index=False)
                utils.logger.info(f"Results saved to {os.path.relpath(experiment_path)}/results.csv")
    return 0


if __name__ == "__main__":
    sys.exit(main())
