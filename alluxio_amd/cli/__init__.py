"""Command-line tools: ``alluxio`` launcher, fs / fsadmin / job shells, runTests, readJournal,
validateEnv / validateConf (reference bin/alluxio, shell/, integration/tools/validation)."""
