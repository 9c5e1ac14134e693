/* placeholder, filled in with kernel 2 */
