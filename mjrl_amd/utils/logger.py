"""DataLog — key -> list store with CSV / pickle dumps (API of mjrl/utils/logger.py:10-57).
Host-side bookkeeping; the update fills it with the same keys as the reference."""
import ast
import csv
import os
import pickle


class DataLog:
    def __init__(self):
        self.log = {}
        self.max_len = 0

    def log_kv(self, key, value):
        self.log.setdefault(key, []).append(value)
        if len(self.log[key]) > self.max_len:
            self.max_len = self.max_len + 1

    def save_log(self, save_path):
        with open(os.path.join(save_path, "log.pickle"), "wb") as f:
            pickle.dump(self.log, f)
        with open(os.path.join(save_path, "log.csv"), "w") as csv_file:
            writer = csv.DictWriter(csv_file, fieldnames=list(self.log.keys()))
            writer.writeheader()
            for row in range(self.max_len):
                writer.writerow({k: v[row] for k, v in self.log.items() if row < len(v)})

    def get_current_log(self):
        return {k: v[-1] for k, v in self.log.items()}

    def read_log(self, log_path):
        """Reloads a log.csv (values parsed as Python literals, never eval'd code)."""
        with open(log_path) as csv_file:
            reader = csv.DictReader(csv_file)
            rows = list(reader)
            data = {k: [] for k in reader.fieldnames}
        for row in rows:
            for k in data:
                try:
                    data[k].append(ast.literal_eval(row[k]))
                except (ValueError, SyntaxError):
                    pass
        self.log = data
